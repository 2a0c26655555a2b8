"""ctypes binding of libcapmi.so (C ABI declared in include/capmi.h).

The library is the only compute path for CUDA(HIP) tensors: there is no
fallback. If it is missing this module raises at import time.

``import torch`` happens first on purpose: torch's bundled libamdhip64.so
(SONAME libamdhip64.so.7) must be the HIP runtime libcapmi binds to, so both
share one runtime (streams, allocations, graph capture).
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libcapmi)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CAPMI_LIB") or os.path.join(_HERE, "libcapmi.so")  # CAPMI_LIB: kernel A/B builds

c_int, c_ll, c_float, c_double, c_vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_double, ctypes.c_void_p
c_ull = ctypes.c_ulonglong

CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_A_CONV_NHWC, CAPMI_A_CONV_NCHW, CAPMI_A_CONV_NHWC4 = 0, 1, 2, 3, 4
CAPMI_B_NMAJOR_W, CAPMI_B_KROWS, CAPMI_B_CONV_NHWC = 0, 1, 2
CAPMI_TILE_128, CAPMI_TILE_64, CAPMI_TILE_128x64, CAPMI_TILE_AUTO, CAPMI_TILE_128_W8 = 0, 1, 2, 3, 4
CAPMI_MAX_GROUP = 4
CAPMI_COLSUM_GROUPS = 64
ABI_VERSION = 26
CAPMI_BNB_RELU_Y, CAPMI_BNB_RELU_OUT = 0, 1
CAPMI_BNB_MAX_SLABS = 256
CAPMI_GEMM_BF16 = 1
CAPMI_GEMM_BF16_IO = 2
CAPMI_GEMM_X3 = 4
CAPMI_GEMM_X3P = 8
CAPMI_GEMM_SPLIT3 = 16
CAPMI_GEMM_X3D = 32
CAPMI_GEMM_X3S = 64
CAPMI_GEMM_X3W = 128
CAPMI_GEMM_X3C = 256


class GemmProblem(ctypes.Structure):
    """Mirror of ``capmi_gemm_problem`` (include/capmi.h)."""
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int), ("ksplit", c_int),
        ("A", c_vp), ("lda", c_ll), ("a_r1", c_ll), ("a_s2", c_ll),
        ("B", c_vp), ("ldb", c_ll),
        ("C", c_vp), ("ldc", c_ll), ("c_r1", c_ll), ("c_s2", c_ll), ("c_split_stride", c_ll),
        ("bias", c_vp), ("bias2", c_vp), ("alpha_ptr", c_vp),
        ("alpha", c_float), ("beta", c_float), ("relu", c_int),
        ("stats", c_vp),
        ("cN", c_int), ("cH", c_int), ("cW", c_int), ("cCin", c_int), ("cKH", c_int),
        ("cKW", c_int), ("cStride", c_int), ("cPad", c_int), ("cHo", c_int), ("cWo", c_int),
        ("in_scale", c_vp), ("in_shift", c_vp),
    ]


class Wx3Job(ctypes.Structure):
    """Mirror of ``capmi_wx3_job`` (include/capmi.h)."""
    _fields_ = [("w", c_vp), ("out", c_vp), ("mode", c_int), ("cout", c_int), ("cin", c_int), ("kh", c_int),
                ("kw", c_int), ("ph", c_int), ("pw", c_int), ("pad_", c_int)]


class DstepSeg(ctypes.Structure):
    """Mirror of ``capmi_dstep_seg`` (include/capmi.h)."""
    _fields_ = [("A", c_vp), ("lda", c_ll), ("W", c_vp), ("ldw", c_ll), ("K", c_int)]


class DstepEpi(ctypes.Structure):
    """Mirror of ``capmi_dstep_epi`` (include/capmi.h)."""
    _fields_ = [
        ("mode", c_int), ("out0", c_vp), ("ld0", c_ll), ("bias0", c_vp), ("nsplit", c_int),
        ("out1", c_vp), ("ld1", c_ll), ("bias1", c_vp), ("act1", c_int), ("D", c_int),
        ("xemb", c_vp), ("c_prev", c_vp), ("h_out", c_vp), ("c_out", c_vp), ("act_out", c_vp),
        ("dhd", c_vp), ("dc_in", c_vp), ("act", c_vp), ("c_cur", c_vp), ("dgates", c_vp), ("dc_out", c_vp),
        ("bt", c_int), ("gate", c_vp), ("awe", c_vp), ("dawe_out", c_vp), ("dgp", c_vp),
    ]


CAPMI_DSTEP_STORE2, CAPMI_DSTEP_LSTM_FWD, CAPMI_DSTEP_LSTM_BWD, CAPMI_DSTEP_GATE_BWD = 0, 1, 2, 3

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "capmi_gemm": [ctypes.POINTER(GemmProblem), c_int, c_int, c_int, c_int, c_vp],
    "capmi_gemm_stat_tiles": [c_int, c_int],
    "capmi_gemm_workspace_bytes": [],
    "capmi_gemm_workspace_flag_bytes": [],
    "capmi_gemm_sk": [ctypes.POINTER(GemmProblem), c_int, c_int, c_int, c_vp, c_ll, c_vp],
    "capmi_gemm_ex": [ctypes.POINTER(GemmProblem), c_int, c_int, c_int, c_int, c_int, c_vp],
    "capmi_gemm_sk_ex": [ctypes.POINTER(GemmProblem), c_int, c_int, c_int, c_int, c_vp, c_ll, c_vp],
    "capmi_gemm_sk_plan": [ctypes.POINTER(GemmProblem), c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp],
    "capmi_last_launch_name": [ctypes.c_char_p, c_int],
    "capmi_splitk_reduce": [c_vp, c_int, c_ll, c_int, c_int, c_ll, c_vp, c_vp, c_ll, c_vp],
    "capmi_colsum": [c_vp, c_int, c_int, c_ll, c_float, c_vp, c_vp, c_int, c_vp],
    "capmi_conv_weight_pack": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_conv_weight_pack_pad": [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_image_nhwc4": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_bn_finalize": [c_vp, c_int, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_float, c_float,
                          c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "capmi_bn_eval_params": [c_vp, c_vp, c_vp, c_vp, c_int, c_float, c_vp, c_vp, c_vp],
    "capmi_bn_add_relu": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_vp],
    "capmi_bn_relu_maxpool": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "capmi_adaptive_avgpool_nhwc": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_conv_weight_pack_dgrad": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_conv_weight_pack_dgrad_s2": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_conv_weight_pack_dgrad_x3": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_weight_x3_batch": [c_vp, c_int, c_ll, c_vp],
    "capmi_conv_weight_unpack": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_zero_upsample2_nhwc": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_bn_bwd_reduce": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_ll, c_int,
                            c_vp, c_vp, c_int, c_vp, c_vp, c_vp],
    "capmi_bn_bwd_apply": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_vp, c_vp],
    "capmi_adaptive_avgpool_bwd_nhwc": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_embed_gather": [c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_ll, c_vp],
    "capmi_embed_dense": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_ll, c_vp],
    "capmi_mean_rows": [c_vp, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_att_score_fwd": [c_vp, c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                            c_vp, c_vp],
    "capmi_att_softmax_ctx_fwd": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_ll, c_vp, c_vp,
                                  c_int, c_ll, c_vp, c_vp, c_vp, c_ll, c_vp],
    "capmi_lstm_cell_fwd": [c_vp, c_int, c_ll, c_vp, c_vp, c_int, c_ll, c_vp, c_int, c_int, c_vp,
                            c_vp, c_vp, c_vp],
    "capmi_dropout": [c_vp, c_ll, c_float, c_ull, c_vp, c_vp, c_vp],
    "capmi_counter_add": [c_vp, c_ll, c_vp],
    "capmi_mask_rows_tb": [c_vp, c_vp, c_int, c_int, c_int, c_ll, c_ll, c_ll, c_vp],
    "capmi_ce_fwd_bwd": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp,
                         c_int, c_vp, c_vp],
    "capmi_alpha_reg_parts": [c_int, c_int],
    "capmi_alpha_reg": [c_vp, c_int, c_int, c_int, c_float, c_vp, c_vp, c_vp],
    "capmi_loss_finalize": [c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp],
    "capmi_lstm_cell_bwd": [c_vp, c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                            c_vp, c_vp, c_vp],
    "capmi_att_alpha_expand": [c_vp, c_ll, c_int, c_int, c_vp, c_vp],
    "capmi_att_dup_pick": [c_vp, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_att_ctx_bwd": [c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp],
    "capmi_att_enc_dinput": [c_vp, c_ll, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_att_score_bwd": [c_vp, c_vp, c_ll, c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                            c_int, c_vp, c_vp, c_vp],
    "capmi_att_enc_grad": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                           ctypes.POINTER(c_int), c_vp],
    "capmi_dstep_gemm": [ctypes.POINTER(DstepSeg), c_int, c_int, c_int, c_int, c_int, c_int,
                         ctypes.POINTER(DstepEpi), c_vp, c_ll, c_vp, c_int, c_vp],
    "capmi_att_fwd_fused": [c_vp, c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_vp, c_vp,
                            c_int, c_int, c_int, c_int, c_int, c_vp, c_ll, c_vp, c_vp, c_ll, c_vp],
    "capmi_att_bwd_fused": [c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_ll, c_vp, c_vp,
                            c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp],
    "capmi_adam_clamp": [c_vp, c_vp, c_vp, c_vp, c_ll, c_double, c_double, c_double, c_double, c_double,
                         c_double, c_double, c_vp, c_vp],
    "capmi_adam_clamp_f64": [c_vp, c_vp, c_vp, c_vp, c_ll, c_double, c_double, c_double, c_double,
                             c_double, c_double, c_double, c_vp, c_vp],
    "capmi_embed_scatter_add": [c_vp, c_ll, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp],
    "capmi_bn_relu_bf16": [c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_vp],
    "capmi_bn_add_relu_bf16": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_vp],
    "capmi_f32_to_bf16": [c_vp, c_ll, c_vp, c_vp],
    "capmi_adaptive_avgpool_bf16": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "capmi_resize_normalize_u8": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                  c_vp, c_vp],
    "capmi_resize_taps_max": [c_int, c_int],
    "capmi_split3_bf16": [c_vp, c_ll, c_vp, c_vp],
    "capmi_bn_relu_split3": [c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_vp],
    "capmi_timing_event_create": [ctypes.POINTER(c_vp)],
    "capmi_timing_event_destroy": [c_vp],
    "capmi_timing_event_record": [c_vp, c_vp],
    "capmi_timing_elapsed_ms": [c_vp, c_vp, ctypes.POINTER(c_float)],
    "capmi_timing_arm": [c_vp, c_vp],
    "capmi_timing_disarm": [],
    "capmi_strerror": [c_int],
    "capmi_abi_version": [],
}
_RESTYPES = {"capmi_strerror": ctypes.c_char_p, "capmi_gemm_workspace_bytes": c_ll,
             "capmi_gemm_workspace_flag_bytes": c_ll}
EXPORTS = tuple(_SIGS)


class CapmiError(RuntimeError):
    pass


def _load(path=LIB_PATH):
    """Bind libcapmi.so at ``path`` (the in-tree build; tools load A/B builds side by side through it)."""
    if not os.path.exists(path):
        raise ImportError(
            f"libcapmi.so not found at {path}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (the HIP kernels are the only "
            "compute path; there is no fallback)")
    lib = ctypes.CDLL(path)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, c_int)
    if lib.capmi_abi_version() != ABI_VERSION:
        raise ImportError("libcapmi.so ABI version mismatch; rebuild it")
    return lib


lib = _load()


def check(code, what=""):
    if code != 0:
        raise CapmiError(f"{what}: {lib.capmi_strerror(code).decode()} (code {code})")


def call(name, *args):
    check(getattr(lib, name)(*args), name)
