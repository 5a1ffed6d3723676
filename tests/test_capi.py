"""The C-ABI library builds, loads without a GPU and exports every symbol include/l3u.h declares;
the ctypes signature table matches the header (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "l3u.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    funcs = {}
    for m in re.finditer(r"\bint\s+(l3u_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        funcs[m.group(1)] = args
    return funcs


def test_header_parses():
    f = header_functions()
    assert "l3u_dw3_fwd" in f and "l3u_pw_fwd" in f and "l3u_ftl_bwd" in f
    assert len(f) >= 25


def test_library_exports_every_header_symbol():
    from light_unet import _native
    lib = _native.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    # and nothing is bound that the header does not declare
    assert set(_native.exported_symbols()) == set(header_functions())


def test_ctypes_signatures_match_header():
    from light_unet import _native
    hf = header_functions()
    kind = {"P": ctypes.c_void_p, "I": ctypes.c_int, "L": ctypes.c_longlong,
            "F": ctypes.c_float, "D": ctypes.c_double, "U": ctypes.c_ulonglong}

    def ctype_of(decl):
        d = decl.replace("const ", "").strip()
        if "*" in d or d.startswith("hipStream_t"):
            return kind["P"]
        t = d.rsplit(" ", 1)[0].strip()
        return {"int": kind["I"], "long long": kind["L"], "float": kind["F"], "double": kind["D"],
                "unsigned long long": kind["U"]}[t]

    for name, args in hf.items():
        bound = _native._SIGS[name]
        assert len(bound) == len(args), name
        for a, b in zip(args, bound):
            assert ctype_of(a) is b, (name, a, b)


def test_bf16_twins_mirror_fp32_entry_points():
    """Every _bf16 twin takes the fp32 entry point's arguments, with some float pointers (the
    activations) as l3u_bf16 pointers and nothing else changed (fp32 and bf16)."""
    from light_unet import _native
    hf = header_functions()
    twins = [n for n in hf if n.endswith("_bf16") and n != "l3u_cast_f32_bf16"]
    assert sorted(twins) == sorted(n + "_bf16" for n in _native.BF16_TWINS)
    for t in twins:
        a32, a16 = hf[t[:-5]], hf[t]
        assert len(a32) == len(a16), t
        nb = 0
        for x, y in zip(a32, a16):
            if x != y:
                assert x.replace("float*", "l3u_bf16*") == y, (t, x, y)
                nb += 1
        # the args-struct entry points (void* activations) differ only in the name
        assert nb >= 1 or "_args*" in a32[0], t


def test_host_queries_without_gpu():
    from light_unet import _native
    assert _native.query("l3u_abi_version") == _native.ABI_VERSION == 5
    assert _native.query("l3u_dw3_nchunk", 4, 32, 48, 48, 48) == 30   # 3 z-slabs x 10 y-strips
    assert _native.query("l3u_dw3_nchunk", 4, 16, 48, 48, 48) == 40   # 12-plane slabs: 4 x 10
    assert _native.query("l3u_pw_bwd_supported", 16, 32, 48 ** 3) == 1
    assert _native.query("l3u_pw_bwd_supported", 32, 64, 24 ** 3) == 1
    assert _native.query("l3u_pw_bwd_supported", 64, 32, 12 ** 3) == 1     # wide form
    assert _native.query("l3u_pw_bwd_supported", 128, 256, 6 ** 3) == 1
    assert _native.query("l3u_pw_bwd_supported", 48, 32, 12 ** 3) == 0
    assert _native.query("l3u_pw_bwd_supported", 16, 128, 12 ** 3) == 0
    assert _native.query("l3u_pw_bwd_supported", 16, 16, 6 * 6 * 7 + 1) == 0
    assert _native.query("l3u_pw_bwd_nparts", 4, 16, 32, 48 ** 3) == \
        _native.query("l3u_pw_bwd_weight_nparts", 4, 48 ** 3)
    assert _native.query("l3u_pw_bwd_nparts", 4, 64, 128, 12 ** 3) == 4 * 27
    assert _native.query("l3u_pw_bwd_nparts", 4, 48, 32, 12 ** 3) == 0
    # the one-read tile kernel: one partial per tile group (12^3: 64-pair tiles, 24^3: 32-pair
    # tiles, two per workgroup)
    assert _native.query("l3u_convt_bwd_fused_nparts", 4, 64, 32, 12, 12, 12) == 4 * 14
    assert _native.query("l3u_convt_bwd_fused_nparts", 4, 32, 16, 24, 24, 24) == 4 * 108
    assert _native.query("l3u_convt_bwd_fused_nparts", 4, 128, 64, 6, 6, 6) == 0
    assert _native.query("l3u_convt_bwd_fused_nparts", 4, 128, 64, 16, 16, 16) == 4 * 8
    assert _native.query("l3u_convt_bwd_fused_nparts", 4, 256, 128, 6, 6, 6) == 0
    # the tile kernel reads dY through a buffer descriptor over one sample: Co * 8 * S floats
    # must stay below 2^31 bytes (Co = 32: S < 2^21), larger volumes take the three-launch path
    assert _native.query("l3u_convt_bwd_fused_nparts", 1, 64, 32, 127, 128, 128) > 0
    assert _native.query("l3u_convt_bwd_fused_nparts", 1, 64, 32, 128, 128, 128) == 0
    assert _native.query("l3u_convt_bwd_fused_nparts", 1, 128, 64, 64, 128, 128) == 0
    assert _native.query("l3u_convt_bwd_fused_nparts", 1, 128, 64, 62, 128, 128) > 0
    assert _native.query("l3u_dw3_nchunk", 4, 32, 24, 24, 24) == 18   # 6 z-slabs x 3 y-strips
    assert _native.query("l3u_dw3_nchunk", 4, 128, 6, 6, 6) == 1
    assert _native.query("l3u_pw_stat_nsb", 16, 16, 48 ** 3) == 432   # 256-voxel tiles


def test_pw_bwd_chunk_invariant():
    """The pointwise-backward voxel chunk and the partial counts agree, for every volume the
    engine can see (csrc/pwconv.hip pw_chunk_ok): each chunk is ONE workgroup sweep -- a multiple
    of 256 voxels (the K = 1 kernel's SCH / 4 threads are whole waves) and at most 512 (its
    128-thread bound) -- and the partial count is N * ceil(S / chunk) for both the fused and the
    weight-only forms.  Round 5's 192-voxel chunks broke the first condition (48-thread
    workgroups) and gave NaN weight gradients; this fails before any GPU run would."""
    from light_unet import _native
    sizes = sorted({d * h * w for d in (3, 4, 5, 6, 8, 11, 12, 16, 24, 32, 40, 48, 64, 80, 128)
                    for h, w in ((d, d), (44, 36), (80, 80), (6, 8))} | {4, 1020, 1024, 4092, 4096,
                                                                        65532, 65536, 256 ** 3})
    for S in sizes:
        ch = _native.query("l3u_pw_bwd_chunk", S)
        assert ch % 256 == 0 and 256 <= ch <= 512, (S, ch)
        for N in (1, 4):
            nsc = -(-S // ch)
            assert _native.query("l3u_pw_bwd_weight_nparts", N, S) == N * nsc, (S, N)
            if S % 4 == 0:
                for J, K in ((16, 1), (16, 16), (32, 16), (16, 32), (32, 64)):
                    assert _native.query("l3u_pw_bwd_nparts", N, J, K, S) == N * nsc, (S, J, K)
    assert _native.query("l3u_pw_bwd_chunk", 0) == 0


def test_no_cpu_fallback_in_product_package():
    """The product package never imports the oracle."""
    pkg = os.path.join(ROOT, "light-3d-unet-front_amd", "light_unet")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f


def test_require_device_rejects_cpu():
    import torch
    from light_unet import _native
    with pytest.raises(_native.NativeError):
        _native.require_device(torch.zeros(3))
