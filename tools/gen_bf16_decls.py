"""Regenerates the bf16-twin block of include/l3u.h from the L3U_TWIN parameter macros in
light-3d-unet-front_amd/csrc/*.hip (the single source of both twins' argument lists), so the
header and the library cannot drift apart (tests/test_capi.py checks the result)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARK = "/* ---- bf16 twins (BASELINE config 3)"
HEAD = MARK + ''' --------------------------------------------------------
 * The same calls with the saved activations (forward inputs and outputs: what the backward
 * re-reads) stored as bf16; argument order and meaning are those of the fp32 entry point without
 * the suffix.  Gradients (every backward input/output gradient), weights, biases, InstanceNorm
 * records and the statistics / weight-gradient partials stay fp32 (fp64 where marked), and every
 * kernel computes in fp32 (bf16 loads widen exactly, stores round to nearest even).
 * l3u_outconv_* keep p / dp / t fp32 (the loss runs on fp32 probabilities); l3u_front_fwd reads
 * the caller's fp32 x and can write its bf16 copy (x_copy) for the backward.  l3u_maxpool2_bwd
 * has no bf16 twin: it reads no saved activation.                                          */
'''


def twins():
    decls = []
    for f in sorted(glob.glob(os.path.join(ROOT, "light-3d-unet-front_amd", "csrc", "*.hip"))):
        s = open(f).read()
        macros = {}
        for m in re.finditer(r"#define (P_\w+)\(TT\) (\((?:[^()]|\([^()]*\))*\))", s, re.S):
            macros[m.group(1)] = re.sub(r"\s*\\\n\s*", " ", m.group(2))
        for m in re.finditer(r"L3U_TWIN\((\w+), (P_\w+),", s):
            decls.append((m.group(1), re.sub(r"\s+", " ", macros[m.group(2)].replace("TT", "l3u_bf16"))))
    return decls


def wrap(name, params):
    head = "int %s_bf16" % name
    parts = [p.strip() for p in params[1:-1].split(",")]
    lines, cur, indent = [], head + "(", " " * (len(head) + 1)
    for k, p in enumerate(parts):
        tok = p + (", " if k < len(parts) - 1 else ");")
        if len(cur) + len(tok.rstrip()) > 100:
            lines.append(cur.rstrip())
            cur = indent
        cur += tok
    lines.append(cur)
    return "\n".join(lines)


def main():
    path = os.path.join(ROOT, "include", "l3u.h")
    h = open(path).read()
    i = h.index(MARK)
    j = h.index("#ifdef __cplusplus\n}\n#endif")
    block = HEAD + "\n".join(wrap(n, p) for n, p in twins()) + "\n\n"
    open(path, "w").write(h[:i] + block + h[j:])


if __name__ == "__main__":
    main()
