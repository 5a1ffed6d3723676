"""ctypes binding of the gfx950 C-ABI library (include/l3u.h -> lib/libl3u_hip.so).

This is the only place the host mirror touches native code.  There is no fallback: if the
library is missing or the tensors are not on a ROCm device, calls raise immediately.
"""
import ctypes
import os
import warnings

import torch  # noqa: F401  (loads the HIP runtime the library binds to: one runtime per process)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "L3U_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libl3u_hip.so"))

# include/l3u.h L3U_ABI_VERSION: the library must report exactly this
ABI_VERSION = 5

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double
U64 = ctypes.c_ulonglong

# name -> argtypes (stream is always the trailing void*; every function returns int hipError_t)
_SIGS = {
    "l3u_abi_version": [],
    "l3u_dw3_nchunk": [I, I, I, I, I],
    "l3u_dw3_fwd": [P, L, P, P, P, P, L, I, I, I, I, I, P],
    "l3u_dw3_bwd": [P, L, P, L, P, P, P, L, I, P, P, I, I, I, I, I, P],
    "l3u_pw_stat_nsb": [I, I, I],
    "l3u_pw_fwd": [P, L, P, I, P, P, L, I, P, I, I, I, I, P],
    "l3u_pw_bwd_weight_nparts": [I, I],
    "l3u_pw_bwd_chunk": [I],
    "l3u_pw_bwd_weight": [P, L, P, L, P, I, I, I, I, P],
    "l3u_pw_bwd_supported": [I, I, I],
    "l3u_pw_bwd_nparts": [I, I, I, I],
    "l3u_pw_bwd": [P, L, P, L, P, P, I, P, L, P, P, L, I, P, I, I, I, I, P],
    "l3u_pw_bwd2_supported": [I, I],
    "l3u_pw_bwd_tail_pair": [P, L, P, P, L, P, I, I, P, L, P, I, P, L, P, P, L, P, P, L, I, P, I, I,
                             P, L, P, P, L, P, P, L, I, P, I, I, I, I, I, P],
    "l3u_pw_bwd2": [P, L, P, L, P, P, L, I, P, I, P, L, P, L, P, P, L, I, P, I, I, I, I, P],
    "l3u_in_finalize": [P, I, P, P, F, U64, P, I, P, I, I, P],
    "l3u_norm_act_nblocks": [I],
    "l3u_norm_act_fwd": [P, L, P, P, P, L, P, P, I, P, L, I, I, I, P],
    "l3u_norm_act_pool_fwd": [P, L, P, P, P, L, P, P, I, P, L, P, L, P, I, I, I, I, I, P],
    "l3u_norm_act_bwd_reduce": [P, L, P, L, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_norm_act_bwd_apply": [P, L, P, L, P, L, P, P, L, P, P, P, L, P, L, I, I, I, P],
    "l3u_in_bwd_apply": [P, L, P, L, P, P, I, P, L, I, I, I, P],
    "l3u_maxpool2_fwd": [P, L, P, L, P, I, I, I, I, I, P],
    "l3u_maxpool2_bwd": [P, L, P, P, L, P, L, I, I, I, I, I, P],
    "l3u_convt_fwd": [P, L, P, P, P, L, I, I, I, I, I, I, P],
    "l3u_convt_bwd": [P, L, P, L, P, P, L, P, P, I, I, I, I, I, I, P],
    "l3u_convt_bwd_fused_nparts": [I, I, I, I, I, I],
    "l3u_convt_bwd_fused": [P, L, P, L, P, P, L, P, P, I, I, I, I, I, I, P],
    "l3u_outconv_nblocks": [I],
    "l3u_outconv_fwd": [P, L, P, P, P, P, P, I, I, I, P],
    "l3u_outconv_bwd": [P, P, P, P, D, D, D, D, P, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_outconv_bwd_ftl": [P, P, P, I, D, D, D, D, P, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_ftl_nblocks": [L],
    "l3u_ftl_sums": [P, P, L, P, P, P],
    "l3u_ftl_reduce": [P, I, P, P],
    "l3u_window_gather": [P, I, I, I, P, I, I, I, I, P, P],
    "l3u_window_blend": [P, P, I, P, I, P, I, P, I, I, I, I, I, I, P, P],
    "l3u_ftl_loss": [P, D, D, D, D, P, P],
    "l3u_ftl_bwd": [P, P, L, P, D, D, D, D, P, I, P, P],
    "l3u_reduce_segments": [P, P, I, P, P],
    "l3u_reduce_segments_adamw": [P, P, I, P, P, P, P, P, F, F, F, F, P, F, P, P, P],
    "l3u_pw_fwd2": [P, L, P, P, L, P, P, L, P, P, L, P, I, I, I, I, P],
    "l3u_adamw_tick": [P, P, P, P, L, P, F, F, F, F, P, F, P, P, P],
    "l3u_front_nblocks": [I],
    "l3u_front_fwd": [P, L, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "l3u_pw_bwd_tail": [P, L, P, L, P, L, P, P, I, I, P, L, P, P, L, I, P, I, I, I, I, P],
    "l3u_norm_act_bwd": [P, L, P, L, P, L, P, P, L, P, P, P, L, P, L, I, I, I, P],
    "l3u_norm_act_bwd_up": [P, L, P, L, P, P, L, P, L, P, P, L, P, P, P, L, P, L, I, I, I, I, I, P],
    "l3u_gconv3_nblocks": [I],
    "l3u_gconv3_wgrad_nparts": [I, I],
    "l3u_gconv3_fwd": [P, L, P, P, P, L, P, I, I, I, I, I, I, I, P],
    "l3u_gconv3_bwd_data": [P, L, P, P, P, L, P, L, I, P, I, I, I, I, I, I, I, P],
    "l3u_gconv3_bwd_weight": [P, L, P, L, P, P, I, I, I, I, I, I, I, P],
    "l3u_counter_add": [P, I, P],
    "l3u_cast_f32_bf16": [P, P, L, P],
    "l3u_box_copy": [P, L, I, I, I, P, L, I, I, I, I, I, I, I, I, P],
    "l3u_ccl_nchunks": [L],
    "l3u_aug_patches": [P, I, I, I, I, P, P, P, P, P, P],
    "l3u_ccl_label": [P, F, P, P, P, I, I, I, P],
    "l3u_ccl_stats": [P, P, P, P, I, I, I, I, P],
    "l3u_ccl_pairs": [P, P, I, P, L, P],
    "l3u_ccl_label_b": [P, F, P, P, P, I, I, I, I, P],
    "l3u_ccl_stats_b": [P, P, P, P, I, I, I, I, I, I, P],
    "l3u_cast_bf16_f32": [P, P, L, P],
    "l3u_outconv_bwd_dz": [P, P, P, P, D, D, D, D, P, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_outconv_bwd_ftl_dz": [P, P, P, I, D, D, D, D, P, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_norm_act_bwd_reduce_r1": [P, L, P, P, L, P, L, P, P, L, P, P, I, I, I, P],
    "l3u_pw_bwd_tail_r1": [P, L, P, P, L, P, L, P, P, I, I, P, L, P, P, L, I, P, I, I, I, I, P],
    "l3u_norm_act_bwd_reduce_up": [P, L, P, L, P, P, L, P, L, P, P, L, P, P, I, I, I, I, I, P],
    "l3u_pw_bwd_tail_up": [P, L, P, L, P, P, L, P, L, P, P, I, I, P, L, P, P, L, I, P, I, I, I, I, I, I,
                           P],
    "l3u_dwpw_supported": [I, I, I, I, I, I],
    "l3u_dw3_bwd_rank1": [I, I, I, I, I],
    "l3u_dwpw_stat_nsb": [I, I, I, I, I],
    "l3u_dwpw_fwd": [P, L, P, P, P, P, P, L, P, P, P, L, P, P, L, I, I, I, I, I, I, P],
}
# entry points with a _bf16 twin (same arguments; saved activations stored as bf16, gradients
# fp32, include/l3u.h)
BF16_TWINS = ("l3u_dw3_fwd", "l3u_dw3_bwd", "l3u_pw_fwd", "l3u_pw_fwd2", "l3u_pw_bwd_weight",
              "l3u_pw_bwd", "l3u_pw_bwd2", "l3u_pw_bwd_tail", "l3u_pw_bwd_tail_pair", "l3u_convt_fwd", "l3u_convt_bwd",
              "l3u_convt_bwd_fused", "l3u_norm_act_fwd", "l3u_norm_act_pool_fwd",
              "l3u_norm_act_bwd_reduce", "l3u_norm_act_bwd_apply", "l3u_norm_act_bwd",
              "l3u_in_bwd_apply", "l3u_maxpool2_fwd", "l3u_outconv_fwd", "l3u_outconv_bwd",
              "l3u_outconv_bwd_ftl", "l3u_box_copy",
              "l3u_front_fwd", "l3u_dwpw_fwd", "l3u_outconv_bwd_dz", "l3u_outconv_bwd_ftl_dz",
              "l3u_norm_act_bwd_reduce_r1", "l3u_pw_bwd_tail_r1", "l3u_norm_act_bwd_reduce_up",
              "l3u_pw_bwd_tail_up", "l3u_norm_act_bwd_up")
for _n in BF16_TWINS:
    _SIGS[_n + "_bf16"] = _SIGS[_n]
# query helpers that return a value instead of an error code
_QUERIES = {"l3u_abi_version", "l3u_dw3_nchunk", "l3u_pw_stat_nsb", "l3u_pw_bwd_weight_nparts",
            "l3u_pw_bwd_supported", "l3u_pw_bwd_nparts", "l3u_convt_bwd_fused_nparts",
            "l3u_norm_act_nblocks", "l3u_outconv_nblocks", "l3u_ftl_nblocks",
            "l3u_gconv3_nblocks", "l3u_gconv3_wgrad_nparts", "l3u_front_nblocks",
            "l3u_ccl_nchunks", "l3u_dwpw_supported", "l3u_dwpw_stat_nsb",
            "l3u_dw3_bwd_rank1", "l3u_pw_bwd2_supported", "l3u_pw_bwd_chunk"}

_lib = None


class NativeError(RuntimeError):
    pass


class NormSrc(ctypes.Structure):
    """struct l3u_norm_src (include/l3u.h): where a consumer kernel finalizes an InstanceNorm
    record from.  Pass `norm_src_ptr(s)`; keep the object alive across the call."""
    _fields_ = [("stat_part", P), ("nsb", I), ("layer", I), ("gamma", P), ("beta", P),
                ("drop_p", F), ("seed", U64), ("step", P), ("rec_out", P), ("rank1", P)]


class AugParam(ctypes.Structure):
    """struct l3u_aug_param (include/l3u.h): one training patch's crop and augmentation."""
    _fields_ = [("image", P), ("label", P), ("z0", I), ("y0", I), ("x0", I), ("sd", I), ("sh", I),
                ("sw", I), ("pz", I), ("py", I), ("px", I), ("flip", I), ("rot_a0", I),
                ("rot_a1", I), ("rot_c", D), ("rot_s", D), ("rot_off0", D), ("rot_off1", D),
                ("zoom", I), ("zs", I * 3), ("zst", I * 3), ("zf", D * 3), ("shift_on", I),
                ("shift", F), ("noise_on", I)]


def norm_src_ptr(s):
    """A pointer argument to `s` that keeps `s` alive as long as the argument itself (so a
    recorded call can be re-issued later)."""
    return None if s is None else ctypes.pointer(s)


def load():
    """Load the library (once).  Raises NativeError if it is missing: there is no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"HIP library not found at {LIB_PATH}; build it with `make -C light-3d-unet-front_amd` "
            "(or __graft_entry__.build()).  The Light-3D-U-Net MI355X path has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    # L3U_SKIP_ABI_CHECK=1: an older variant build on purpose (A/B of an earlier commit's csrc/);
    # its missing entry points stay unbound (calling one raises) and a version mismatch only warns
    skip = os.environ.get("L3U_SKIP_ABI_CHECK") == "1"
    for name, args in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None and skip:
            continue
        if fn is None:
            raise NativeError(f"{LIB_PATH} does not export {name}: rebuild the library")
        fn.argtypes = args
        fn.restype = I
    ver = lib.l3u_abi_version()
    if ver != ABI_VERSION:
        msg = (f"{LIB_PATH} reports ABI version {ver}, this binding expects {ABI_VERSION}: "
               "rebuild the library")
        if not skip:
            raise NativeError(msg)
        warnings.warn(msg + " (L3U_SKIP_ABI_CHECK=1: loading it anyway)")
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS)


def query(name, *args):
    return getattr(load(), name)(*args)


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed with hipError {rc}")


def stream():
    return torch.cuda.current_stream().cuda_stream


def ptr(t, offset=0):
    """Device pointer of tensor `t` (+ element offset).  None -> NULL."""
    if t is None:
        return None
    return t.data_ptr() + offset * t.element_size()


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda or t.dtype not in (torch.float32, torch.float64,
                                                               torch.bfloat16, torch.int32,
                                                               torch.int64, torch.uint8)):
            raise NativeError(
                f"light_unet MI355X path needs ROCm device tensors (got {t.device}, {t.dtype}); "
                "there is no CPU fallback")
