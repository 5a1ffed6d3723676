"""Content hash of the product tree: the HIP sources, the C-ABI header and the host package.

Evidence records (tools/instep.py, tools/pmc_*_json.py) store it as "tree"; bench.py computes it
at run time and quotes only the records whose tree equals its own, so a record taken on an older
kernel set is never presented as this step's (the GPU box has no .git, so a commit id cannot be
checked there; the hash can).

    python tools/treehash.py        # prints the hash
"""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-3d-unet-front_amd")


def product_files():
    files = glob.glob(os.path.join(PKG, "csrc", "*"))
    files += glob.glob(os.path.join(PKG, "light_unet", "**", "*.py"), recursive=True)
    files += [os.path.join(ROOT, "include", "l3u.h"), os.path.join(PKG, "Makefile")]
    return sorted(f for f in files if os.path.isfile(f))


def product_tree():
    h = hashlib.sha256()
    for f in product_files():
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(product_tree())
