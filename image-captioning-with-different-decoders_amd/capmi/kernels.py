"""Thin Python wrappers over libcapmi's C ABI (one function per entry point).

Shape/dtype/device validation happens here, before the call (include/capmi.h
contract); every launch goes on ``torch.cuda.current_stream()``.
"""
import ctypes
import weakref

import torch

from ._lib import DstepEpi, DstepSeg
from ._lib import (CAPMI_A_CONV_NHWC, CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_B_NMAJOR_W, CAPMI_BNB_MAX_SLABS, CAPMI_GEMM_BF16,
                   CAPMI_GEMM_BF16_IO, CAPMI_GEMM_X3, CAPMI_GEMM_X3P,
                   CAPMI_GEMM_SPLIT3, CAPMI_GEMM_X3C, CAPMI_GEMM_X3D, CAPMI_GEMM_X3S, CAPMI_GEMM_X3W,
                   CAPMI_COLSUM_GROUPS, CAPMI_TILE_128, CAPMI_TILE_64,
                   CAPMI_TILE_128x64, CAPMI_TILE_AUTO, GemmProblem, call, lib)

F32 = torch.float32


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def _cuda(*ts, dtype=F32):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("capmi kernels need device (HIP) tensors")
        if dtype is not None and t.dtype != dtype:
            raise TypeError(f"expected {dtype}, got {t.dtype}")


# --------------------------------------------------------------------------------------
# GEMM
# --------------------------------------------------------------------------------------
def problem(M, N, K, A, lda, B, ldb, C, ldc, *, a_r1=0, a_s2=0, c_r1=0, c_s2=0, ksplit=1,
            c_split_stride=0, bias=None, bias2=None, alpha=1.0, alpha_ptr=None, beta=0.0,
            relu=False, stats=None, conv=None, in_scale=None, in_shift=None):
    """Build one ``capmi_gemm_problem``. A/B/C are tensors (or views) whose data_ptr is the
    operand origin; ld* are element strides. ``conv`` = dict(N,H,W,Cin,KH,KW,stride,pad,Ho,Wo).
    The problem keeps raw pointers only: the caller holds every tensor until the launch."""
    _cuda(C, bias, bias2, stats, in_scale, in_shift)
    for t_ in (A, B):  # bf16: the split planes of gemm_x3 (B) / gemm_x3p (A and B)
        _cuda(t_, dtype=torch.bfloat16 if t_ is not None and t_.dtype == torch.bfloat16 else F32)
    p = GemmProblem()
    p.M, p.N, p.K, p.ksplit = int(M), int(N), int(K), int(ksplit)
    p.A, p.lda, p.a_r1, p.a_s2 = ptr(A), int(lda), int(a_r1), int(a_s2)
    p.B, p.ldb = ptr(B), int(ldb)
    p.C, p.ldc, p.c_r1, p.c_s2, p.c_split_stride = ptr(C), int(ldc), int(c_r1), int(c_s2), int(c_split_stride)
    p.bias, p.bias2 = ptr(bias), ptr(bias2)
    p.alpha_ptr = ptr(alpha_ptr)
    p.alpha, p.beta, p.relu = float(alpha), float(beta), int(bool(relu))
    p.stats = ptr(stats)
    if conv is not None:
        p.cN, p.cH, p.cW, p.cCin = conv["N"], conv["H"], conv["W"], conv["Cin"]
        p.cKH, p.cKW, p.cStride, p.cPad = conv["KH"], conv["KW"], conv["stride"], conv["pad"]
        p.cHo, p.cWo = conv["Ho"], conv["Wo"]
    p.in_scale, p.in_shift = ptr(in_scale), ptr(in_shift)
    return p


def gemm(problems, amode=CAPMI_A_KMAJOR, bmode=CAPMI_B_NMAJOR_W, tile=CAPMI_TILE_128, flags=0):
    """flags: 0 (fp32 MFMA), CAPMI_GEMM_BF16 (bf16 operands) or CAPMI_GEMM_SPLIT3 (fp32-accurate
    three-term split on the bf16 matrix cores; capmi_gemm_ex)."""
    if isinstance(problems, GemmProblem):
        problems = [problems]
    arr = (GemmProblem * len(problems))(*problems)
    if flags:
        call("capmi_gemm_ex", arr, len(problems), amode, bmode, tile, flags, stream())
    else:
        call("capmi_gemm", arr, len(problems), amode, bmode, tile, stream())


def gemm_workspace_bytes():
    return int(lib.capmi_gemm_workspace_bytes())


_WORKSPACES = weakref.WeakSet()


def gemm_workspace(device):
    """Zeroed stream-K workspace for capmi_gemm_sk (one per stream that runs it)."""
    n = (gemm_workspace_bytes() + 3) // 4
    ws = torch.zeros(n, device=device, dtype=torch.int32)
    _WORKSPACES.add(ws)
    return ws


def sk_check(workspaces=None):
    """Host-side check of the stream-K hand-off invariant at a sync point: every flag word of a
    workspace is zero between launches (include/capmi.h, capmi_gemm_workspace_flag_bytes). A
    nonzero word means a hand-off timed out and a result is invalid: the flags are re-zeroed (so
    later launches start clean) and RuntimeError is raised. Reads every live workspace by default
    (one small device->host copy each); call it only where the host synchronises anyway."""
    nflag = int(lib.capmi_gemm_workspace_flag_bytes()) // 4
    bad = []
    for ws in list(_WORKSPACES) if workspaces is None else workspaces:
        f = ws[:nflag]
        if bool(f.any()):
            bad.append(int(f.count_nonzero()))
            f.zero_()
    if bad:
        raise RuntimeError(f"capmi stream-K: hand-off timed out ({bad} nonzero flag words); results of the "
                           "launches since the last check are invalid (flags re-zeroed)")


def gemm_sk(prob, amode, workspace, tile=CAPMI_TILE_AUTO, bmode=CAPMI_B_NMAJOR_W, bf16=False, flags=None):
    """bf16: operands rounded to bf16 in LDS, bf16 MFMA with fp32 accumulation (CAPMI_GEMM_BF16).
    flags (overrides bf16): 0, CAPMI_GEMM_BF16 or CAPMI_GEMM_SPLIT3."""
    _cuda(workspace, dtype=torch.int32)
    f = (1 if bf16 else 0) if flags is None else flags
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, bmode, tile, f, ptr(workspace),
         workspace.numel() * 4, stream())


def problem_bf16(M, N, K, A, lda, B, ldb, C, ldc, *, stats=None, conv=None):
    """capmi_gemm_problem over bf16 A / B / C (CAPMI_GEMM_BF16_IO): plain conv or dense GEMM,
    fp32 BN statistics of the stored (bf16) output."""
    _cuda(A, B, C, dtype=torch.bfloat16)
    _cuda(stats)
    p = GemmProblem()
    p.M, p.N, p.K, p.ksplit = int(M), int(N), int(K), 1
    p.A, p.lda, p.B, p.ldb = ptr(A), int(lda), ptr(B), int(ldb)
    p.C, p.ldc = ptr(C), int(ldc)
    p.alpha, p.beta = 1.0, 0.0
    p.stats = ptr(stats)
    if conv is not None:
        p.cN, p.cH, p.cW, p.cCin = conv["N"], conv["H"], conv["W"], conv["Cin"]
        p.cKH, p.cKW, p.cStride, p.cPad = conv["KH"], conv["KW"], conv["stride"], conv["pad"]
        p.cHo, p.cWo = conv["Ho"], conv["Wo"]
    return p


def gemm_bf16(prob, amode, workspace, tile=CAPMI_TILE_AUTO):
    """bf16-in / bf16-out GEMM or implicit-GEMM conv (CAPMI_GEMM_BF16_IO)."""
    _cuda(workspace, dtype=torch.int32)
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, tile, CAPMI_GEMM_BF16_IO,
         ptr(workspace), workspace.numel() * 4, stream())


def split3_bf16(w, out):
    """fp32 ``w`` (numel % 4 == 0) -> ``out`` bf16 [3][numel]: the exact three-term split (B operand
    of gemm_x3)."""
    _cuda(w)
    _cuda(out, dtype=torch.bfloat16)
    if out.numel() < 3 * w.numel():
        raise ValueError("split3_bf16: out needs 3 * numel elements")
    call("capmi_split3_bf16", ptr(w), w.numel(), ptr(out), stream())


def gemm_x3(prob, amode, workspace, tile=CAPMI_TILE_AUTO):
    """fp32-accurate GEMM on the bf16 matrix cores (CAPMI_GEMM_X3): fp32 A x B pre-split by
    split3_bf16 (prob.B = plane 0, prob.ldb its row stride)."""
    _cuda(workspace, dtype=torch.int32)
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, tile, CAPMI_GEMM_X3,
         ptr(workspace), workspace.numel() * 4, stream())


def bn_relu_split3(y, scale, shift, rows, C, out):
    """out[3][rows*C] bf16 = the exact split of relu(y*scale+shift) (scale None: of y)."""
    _cuda(y, scale, shift)
    _cuda(out, dtype=torch.bfloat16)
    if out.numel() < 3 * rows * C:
        raise ValueError("bn_relu_split3: out needs 3 * rows * C elements")
    call("capmi_bn_relu_split3", ptr(y), ptr(scale), ptr(shift), int(rows), int(C), ptr(out), stream())


def conv_weight_order_x3p(w, KH, KW, Cin):
    """Packed conv weight [Cout][KH][KW][Cin] (or [Cout][K]) -> the k order of the x3p conv GEMM,
    (ci / 32, kh, kw, ci % 32): the taps of one 32-channel slice consecutive (gemm_x3p.hip)."""
    Cout = w.shape[0]
    if KH * KW == 1:
        return w.reshape(Cout, -1)
    return w.reshape(Cout, KH, KW, Cin // 32, 32).permute(0, 3, 1, 2, 4).reshape(Cout, KH * KW * Cin)


def gemm_x3p(prob, amode, workspace):
    """CAPMI_GEMM_X3P: A (prob.A) and B (prob.B) are both plane 0 of three bf16 split planes."""
    _cuda(workspace, dtype=torch.int32)
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3P,
         ptr(workspace), workspace.numel() * 4, stream())


def gemm_x3d(prob, amode, workspace):
    """CAPMI_GEMM_X3D: A fp32 (dense, or the NHWC conv input with the optional BN prologue) split
    in-kernel x B = three bf16 planes in the x3p k order (conv_weight_order_x3p + split3_bf16)."""
    _cuda(workspace, dtype=torch.int32)
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3D,
         ptr(workspace), workspace.numel() * 4, stream())


def gemm_x3s(prob, amode):
    """CAPMI_GEMM_X3S: the K = 64 convs (dense rows, or a 1x1 conv input with the optional BN prologue) x
    B = three bf16 planes (split3_bf16), store-only epilogue; persistent, no workspace."""
    call("capmi_gemm_sk_ex", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3S,
         None, 0, stream())


def gemm_x3c(prob):
    """CAPMI_GEMM_X3C: the direct 3x3 / stride-1 conv (N = 64, Cin % 32 == 0, W <= 64, the staged band within LDS, optional BN prologue) x
    B = three bf16 planes in the x3p k order; store-only epilogue, no workspace."""
    call("capmi_gemm_sk_ex", ctypes.byref(prob), CAPMI_A_CONV_NHWC, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3C,
         None, 0, stream())


def gemm_x3c_ok(prob):
    """True when CAPMI_GEMM_X3C takes this conv problem (its planner accepts it)."""
    v = [ctypes.c_int(0) for _ in range(5)]
    return lib.capmi_gemm_sk_plan(ctypes.byref(prob), CAPMI_A_CONV_NHWC, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO,
                                  CAPMI_GEMM_X3C, *[ctypes.byref(x) for x in v]) == 0


def gemm_x3c_kernel_name(prob):
    return f"gemm_x3c_kernel<{'true' if prob.in_scale else 'false'}>"


def gemm_x3w(prob, bmode, workspace, bf16=False):
    """CAPMI_GEMM_X3W: the conv weight gradient dW = dY^T . B (A = dY fp32 k rows, CAPMI_A_MMAJOR; B fp32 k
    rows, CAPMI_B_KROWS, or the NHWC conv input's im2col, CAPMI_B_CONV_NHWC, with the optional BN prologue);
    k-split partial slabs in the stream-K workspace. bf16: one bf16 term per operand (| CAPMI_GEMM_BF16, ABI 26)."""
    _cuda(workspace, dtype=torch.int32)
    call("capmi_gemm_sk_ex", ctypes.byref(prob), CAPMI_A_MMAJOR, bmode, CAPMI_TILE_AUTO, _x3w_flags(bf16),
         ptr(workspace), workspace.numel() * 4, stream())


def _x3w_flags(bf16):
    return CAPMI_GEMM_X3W | (CAPMI_GEMM_BF16 if bf16 else 0)


def gemm_x3w_kernel_name(prob, bmode, bf16=False):
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), CAPMI_A_MMAJOR, bmode, CAPMI_TILE_AUTO, _x3w_flags(bf16),
         *[ctypes.byref(x) for x in v])
    return f"{'gemm_w16_kernel' if bf16 else 'gemm_x3w_kernel'}<{bmode}, {'true' if v[2].value else 'false'}>"


def gemm_x3w_ok(prob, bmode, bf16=False):
    """True when CAPMI_GEMM_X3W takes this weight-gradient problem (its planner accepts it)."""
    v = [ctypes.c_int(0) for _ in range(5)]
    return lib.capmi_gemm_sk_plan(ctypes.byref(prob), CAPMI_A_MMAJOR, bmode, CAPMI_TILE_AUTO, _x3w_flags(bf16),
                                  *[ctypes.byref(x) for x in v]) == 0


def gemm_x3s_ok(prob, amode):
    """True when CAPMI_GEMM_X3S takes this problem (its planner accepts it)."""
    v = [ctypes.c_int(0) for _ in range(5)]
    return lib.capmi_gemm_sk_plan(ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3S,
                                  *[ctypes.byref(x) for x in v]) == 0


def gemm_x3s_kernel_name(prob, amode):
    ncb = {64: 1, 128: 2, 256: 4}[prob.N]
    return f"gemm_x3s_kernel<{ncb}, {'true' if prob.in_scale else 'false'}>"


def gemm_x3d_kernel_name(prob, amode):
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3D,
         *[ctypes.byref(x) for x in v])
    b = lambda x: "true" if x else "false"  # noqa: E731
    return f"gemm_x3p_kernel<{amode}, {b(v[2].value)}, 32, true, {b(bool(prob.in_scale))}>"


def gemm_x3p_kernel_name(prob, amode):
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, CAPMI_TILE_AUTO, CAPMI_GEMM_X3P,
         *[ctypes.byref(x) for x in v])
    return f"gemm_x3p_kernel<{amode}, {'true' if v[2].value else 'false'}, {v[3].value}, false, false>"


def gemm_x3_kernel_name(prob, amode, tile=CAPMI_TILE_AUTO):
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, tile, CAPMI_GEMM_X3,
         *[ctypes.byref(x) for x in v])
    b = lambda x: "true" if x else "false"  # noqa: E731
    return f"gemm_x3_kernel<{v[1].value}, {amode}, {b(bool(prob.in_scale))}, {b(v[2].value)}>"


def gemm_bf16_kernel_name(prob, amode, tile=CAPMI_TILE_AUTO):
    """The instantiation gemm_bf16(prob, amode, workspace, tile) launches (capmi_gemm_sk_plan with
    CAPMI_GEMM_BF16_IO: the launcher's own plan, gemm.hip bf16_io_plan)."""
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), amode, CAPMI_B_NMAJOR_W, tile, CAPMI_GEMM_BF16_IO,
         *[ctypes.byref(x) for x in v])
    return f"gemm_bf16_kernel<128, {v[1].value}, {amode}, {'true' if v[2].value else 'false'}, {v[3].value}>"


def last_launch_name():
    """The demangled instantiation of the last GEMM kernel launched on this thread (capmi_last_launch_name)."""
    buf = ctypes.create_string_buffer(512)
    call("capmi_last_launch_name", buf, 512)
    return buf.value.decode()


def gemm_sk_plan(prob, amode, tile=CAPMI_TILE_AUTO, bmode=CAPMI_B_NMAJOR_W, bf16=False, threads=False,
                 flags=None):
    """(bm, bn, stream_k, generic[, threads]) of the launch gemm_sk would make for ``prob``."""
    f = (1 if bf16 else 0) if flags is None else flags
    v = [ctypes.c_int(0) for _ in range(5)]
    call("capmi_gemm_sk_plan", ctypes.byref(prob), amode, bmode, tile, f, *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v[:5 if threads else 4])


def gemm_sk_kernel_name(prob, amode, bmode=CAPMI_B_NMAJOR_W, bf16=False, tile=CAPMI_TILE_AUTO, flags=None):
    """The kernel symbol (as rocprofv3 prints it) of the launch gemm_sk(..., tile) makes."""
    f = (1 if bf16 else 0) if flags is None else flags
    bm, bn, sk, generic, nt = gemm_sk_plan(prob, amode, tile, bmode, threads=True, flags=f)
    b = lambda v: "true" if v else "false"  # noqa: E731
    pro = b(bool(prob.in_scale))
    if generic:
        return "gemm_kernel (generic)"
    if nt == 512:
        return f"gemm_nt8_kernel<{amode}, {pro}, {b(sk)}>"
    split = f == CAPMI_GEMM_SPLIT3 or (f == 1 and (amode == 1 or bmode == 1))
    if split and not (f == 1 and bmode == 0 and amode != 1):
        # rocprofv3 prints the defaulted PRO argument too (true: the BN-prologue conv form)
        return f"gemm_nts_kernel<{bm}, {bn}, {amode}, {bmode}, {b(sk)}, {3 if f == CAPMI_GEMM_SPLIT3 else 1}, {pro}>"
    return f"gemm_nt_kernel<{bm}, {bn}, {amode}, {bmode}, {pro}, {b(sk)}, {b(f == 1)}>"


def stat_tiles(M, tile=CAPMI_TILE_128):
    return lib.capmi_gemm_stat_tiles(int(M), int(tile))


def tiles_for(M, N, tile):
    bm = 64 if tile == CAPMI_TILE_64 else 128
    bn = 128 if tile == CAPMI_TILE_128 else 64
    return ((M + bm - 1) // bm) * ((N + bn - 1) // bn)


def splitk_reduce(inp, S, slab, rows, cols, ld_in, out, ld_out, bias=None):
    _cuda(inp, out, bias)
    call("capmi_splitk_reduce", ptr(inp), S, slab, rows, cols, ld_in, ptr(bias), ptr(out), ld_out,
         stream())


def colsum_work_size(rows, cols):
    return CAPMI_COLSUM_GROUPS * cols


def colsum(inp, rows, cols, ld, out, work, scale=1.0, accumulate=False):
    _cuda(inp, out, work)
    assert work.numel() >= colsum_work_size(rows, cols)
    call("capmi_colsum", ptr(inp), rows, cols, ld, scale, ptr(work), ptr(out), int(accumulate), stream())


# --------------------------------------------------------------------------------------
# encoder
# --------------------------------------------------------------------------------------
def conv_weight_pack(w, out):
    _cuda(w, out)
    co, ci, kh, kw = w.shape
    assert w.is_contiguous() and out.numel() == w.numel()
    call("capmi_conv_weight_pack", ptr(w), co, ci, kh, kw, ptr(out), stream())


def conv_weight_pack_pad(w, cin_pad, out):
    _cuda(w, out)
    co, ci, kh, kw = w.shape
    assert w.is_contiguous() and out.numel() == co * kh * kw * cin_pad
    call("capmi_conv_weight_pack_pad", ptr(w), co, ci, kh, kw, cin_pad, ptr(out), stream())


def image_nhwc4(imgs, out):
    _cuda(imgs, out)
    N, C, H, W = imgs.shape
    assert imgs.is_contiguous() and out.numel() >= N * H * W * 4
    call("capmi_image_nhwc4", ptr(imgs), N, C, H, W, ptr(out), stream())


def bn_work_doubles(C):
    """CAPMI_BN_WORK_DOUBLES: 64 counter doubles + fp64 partials (allocate zeroed)."""
    return 64 + 64 * C


def bn_finalize(stats, tiles, C, count, gamma, beta, running_mean, running_var, momentum, eps,
                scale, shift, work, save_mean=None, save_var=None):
    _cuda(stats, gamma, beta, running_mean, running_var, scale, shift, save_mean, save_var)
    _cuda(work, dtype=torch.float64)
    assert work.numel() >= bn_work_doubles(C)
    call("capmi_bn_finalize", ptr(stats), tiles, C, count, ptr(gamma), ptr(beta), ptr(running_mean),
         ptr(running_var), momentum, eps, ptr(scale), ptr(shift), ptr(save_mean), ptr(save_var),
         ptr(work), stream())


def bn_eval_params(gamma, beta, rm, rv, C, eps, scale, shift):
    _cuda(gamma, beta, rm, rv, scale, shift)
    call("capmi_bn_eval_params", ptr(gamma), ptr(beta), ptr(rm), ptr(rv), C, eps, ptr(scale), ptr(shift),
         stream())


def bn_add_relu(y, s, b, res, out, rows, C, res_scale=None, res_shift=None):
    _cuda(y, s, b, res, out, res_scale, res_shift)
    call("capmi_bn_add_relu", ptr(y), ptr(s), ptr(b), ptr(res), ptr(res_scale), ptr(res_shift),
         ptr(out), rows, C, stream())


def bn_relu_maxpool(y, s, b, out, N, H, W, C, Ho, Wo):
    _cuda(y, s, b, out)
    call("capmi_bn_relu_maxpool", ptr(y), ptr(s), ptr(b), ptr(out), N, H, W, C, Ho, Wo, stream())


def bn_relu_bf16(y, s, b, rows, C, x):
    _cuda(y, x, dtype=torch.bfloat16)
    _cuda(s, b)
    call("capmi_bn_relu_bf16", ptr(y), ptr(s), ptr(b), rows, C, ptr(x), stream())


def bn_add_relu_bf16(y, s, b, res, out, rows, C, res_scale=None, res_shift=None):
    _cuda(y, res, out, dtype=torch.bfloat16)
    _cuda(s, b, res_scale, res_shift)
    call("capmi_bn_add_relu_bf16", ptr(y), ptr(s), ptr(b), ptr(res), ptr(res_scale), ptr(res_shift),
         rows, C, ptr(out), stream())


def f32_to_bf16(x, out):
    _cuda(x)
    _cuda(out, dtype=torch.bfloat16)
    assert x.is_contiguous() and out.numel() >= x.numel()
    call("capmi_f32_to_bf16", ptr(x), x.numel(), ptr(out), stream())


def adaptive_avgpool_bf16(inp, N, H, W, C, OH, OW, out):
    _cuda(inp, dtype=torch.bfloat16)
    _cuda(out)
    call("capmi_adaptive_avgpool_bf16", ptr(inp), N, H, W, C, OH, OW, ptr(out), stream())


def resize_normalize_u8(src, offsets, heights, widths, max_h, max_w, OH, OW, mean, std, tmp, out):
    """Batch of packed uint8 RGB HWC images -> (B, 3, OH, OW) fp32: PIL-exact bilinear Resize,
    ToTensor, Normalize (capmi_resize_normalize_u8). offsets int64 / heights, widths int32 [B] on
    the device; tmp uint8 >= B * max_h * OW * 3."""
    B = heights.numel()
    _cuda(src, tmp, dtype=torch.uint8)
    _cuda(offsets, dtype=torch.int64)
    _cuda(heights, widths, dtype=torch.int32)
    _cuda(out)
    assert tmp.numel() >= B * max_h * OW * 3 and out.numel() >= B * 3 * OH * OW
    m = (ctypes.c_float * 3)(*mean)
    s = (ctypes.c_float * 3)(*std)
    call("capmi_resize_normalize_u8", ptr(src), ptr(offsets), ptr(heights), ptr(widths), B, max_h, max_w, OH, OW,
         m, s, ptr(tmp), ptr(out), stream())


def adaptive_avgpool_nhwc(inp, N, H, W, C, OH, OW, out):
    _cuda(inp, out)
    call("capmi_adaptive_avgpool_nhwc", ptr(inp), N, H, W, C, OH, OW, ptr(out), stream())


# --------------------------------------------------------------------------------------
# encoder fine-tune backward
# --------------------------------------------------------------------------------------
def conv_weight_pack_dgrad(w, out):
    """out[ci][kh][kw][co] = w[co][ci][KH-1-kh][KW-1-kw]"""
    _cuda(w, out)
    co, ci, kh, kw = w.shape
    assert w.is_contiguous() and out.numel() == w.numel()
    call("capmi_conv_weight_pack_dgrad", ptr(w), co, ci, kh, kw, ptr(out), stream())


def conv_weight_pack_dgrad_s2(w, ph, pw, out):
    """3x3 stride-2 conv, parity class (ph, pw): out[ci][th][tw][co] = w[co][ci][kh(th)][kw(tw)],
    kh = 1 (ph = 0) or 2 - 2*th (ph = 1)."""
    _cuda(w, out)
    co, ci, kh, kw = w.shape
    assert (kh, kw) == (3, 3) and w.is_contiguous() and out.numel() >= co * ci * (ph + 1) * (pw + 1)
    call("capmi_conv_weight_pack_dgrad_s2", ptr(w), co, ci, int(ph), int(pw), ptr(out), stream())


WX3_FWD, WX3_FWD_X3P, WX3_DGRAD, WX3_DGRAD_T = 0, 1, 2, 3


def wx3_jobs(specs, device):
    """Device array of capmi_wx3_job descriptors from (w, out, mode, ph, pw) tuples (w: the nn.Conv2d weight,
    out: its [3][R][Kc] bf16 planes); the tensors must outlive every launch of the array."""
    from ._lib import Wx3Job
    arr = (Wx3Job * len(specs))()
    big = 0
    for i, (w, out, mode, ph, pw) in enumerate(specs):
        co, ci, kh, kw = w.shape
        assert w.is_contiguous() and w.dtype == torch.float32 and out.dtype == torch.bfloat16
        T = (ph + 1) * (pw + 1) if mode == WX3_DGRAD and ph >= 0 else kh * kw
        assert out.numel() >= 3 * co * ci * T
        assert mode != WX3_DGRAD_T or kh * kw == 1
        assert mode != WX3_FWD_X3P or ci % 32 == 0
        assert mode != WX3_DGRAD or (co % 32 == 0 and (ph < 0 or (kh == 3 and kw == 3)))
        arr[i] = Wx3Job(w.data_ptr(), out.data_ptr(), mode, co, ci, kh, kw, ph, pw, 0)
        big = max(big, co * ci * T)
        assert big < 2 ** 31  # (the kernel indexes a job's elements in 32 bits)
    raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return raw.to(device), big


def weight_x3_batch(jobs, njobs):
    """capmi_weight_x3_batch: the three-plane splits of every job in ``jobs`` = wx3_jobs(...) (the device
    array and its largest job's element count) in one launch."""
    arr, big = jobs
    _cuda(arr, dtype=torch.uint8)
    call("capmi_weight_x3_batch", ptr(arr), int(njobs), int(big), stream())


def conv_weight_pack_dgrad_x3(w, out, ph=-1, pw=-1):
    """The dgrad weight pack (ph < 0: conv_weight_pack_dgrad; else the sub-pixel class (ph, pw) of
    conv_weight_pack_dgrad_s2) in the x3p conv k order, split into out bf16 [3][Cin][T * Cout]
    (the x3d B operand; == split3_bf16(conv_weight_order_x3p(pack)))."""
    _cuda(w)
    _cuda(out, dtype=torch.bfloat16)
    co, ci, kh, kw = w.shape
    taps = kh * kw if ph < 0 else (ph + 1) * (pw + 1)
    assert w.is_contiguous() and co % 32 == 0 and out.numel() >= 3 * taps * co * ci
    call("capmi_conv_weight_pack_dgrad_x3", ptr(w), co, ci, kh, kw, int(ph), int(pw), ptr(out), stream())


def conv_weight_unpack(packed, shape, out):
    """[Cout][KH][KW][Cin] -> out [Cout][Cin][KH][KW] (``shape`` = nn.Conv2d weight shape)"""
    _cuda(packed, out)
    co, ci, kh, kw = shape
    assert packed.numel() >= co * ci * kh * kw and out.numel() == co * ci * kh * kw and out.is_contiguous()
    call("capmi_conv_weight_unpack", ptr(packed), co, ci, kh, kw, ptr(out), stream())


def zero_upsample2_nhwc(dy, N, Ho, Wo, C, H, W, out):
    _cuda(dy, out)
    assert dy.numel() >= N * Ho * Wo * C and out.numel() >= N * H * W * C
    call("capmi_zero_upsample2_nhwc", ptr(dy), N, Ho, Wo, C, H, W, ptr(out), stream())


def bnb_work_floats(C):
    return 2 * CAPMI_BNB_MAX_SLABS * C


def bn_bwd_reduce(mode, d, y, mask_src, scale, shift, gamma, save_mean, save_var, eps, rows, C, dgamma,
                  dbeta, coef, work, accumulate=False):
    _cuda(d, y, mask_src, scale, shift, gamma, save_mean, save_var, dgamma, dbeta, coef, work)
    assert work.numel() >= bnb_work_floats(C) and coef.numel() >= 4 * C
    assert d.numel() >= rows * C and y.numel() >= rows * C
    call("capmi_bn_bwd_reduce", int(mode), ptr(d), ptr(y), ptr(mask_src), ptr(scale), ptr(shift), ptr(gamma),
         ptr(save_mean), ptr(save_var), float(eps), int(rows), int(C), ptr(dgamma), ptr(dbeta),
         int(bool(accumulate)), ptr(coef), ptr(work), stream())


def bn_bwd_apply(mode, d, y, mask_src, scale, shift, coef, rows, C, dy, dz_out=None):
    _cuda(d, y, mask_src, scale, shift, coef, dy, dz_out)
    assert d.numel() >= rows * C and dy.numel() >= rows * C
    call("capmi_bn_bwd_apply", int(mode), ptr(d), ptr(y), ptr(mask_src), ptr(scale), ptr(shift), ptr(coef),
         int(rows), int(C), ptr(dy), ptr(dz_out), stream())


def adaptive_avgpool_bwd_nhwc(dout, N, H, W, C, OH, OW, din):
    _cuda(dout, din)
    assert dout.numel() >= N * OH * OW * C and din.numel() >= N * H * W * C
    call("capmi_adaptive_avgpool_bwd_nhwc", ptr(dout), N, H, W, C, OH, OW, ptr(din), stream())


# --------------------------------------------------------------------------------------
# decoder
# --------------------------------------------------------------------------------------
def embed_gather(emb, caps, B, L, T, out, ld_out):
    _cuda(emb, dtype=None)
    _cuda(out)
    _cuda(caps, dtype=torch.int64)
    assert emb.dtype in (torch.float32, torch.float64) and emb.is_contiguous() and caps.is_contiguous()
    call("capmi_embed_gather", ptr(emb), int(emb.dtype == torch.float64), emb.shape[1], ptr(caps), B, L,
         T, ptr(out), ld_out, stream())


def embed_dense(emb, T, out, ld_out):
    """emb (B, Le, M) fp32 contiguous -> out[t][b][0:M], t < T"""
    _cuda(emb, out)
    B, Le, M = emb.shape
    assert emb.is_contiguous()
    call("capmi_embed_dense", ptr(emb), B, Le, M, T, ptr(out), ld_out, stream())


def mean_rows(enc, B, P, E, out):
    _cuda(enc, out)
    call("capmi_mean_rows", ptr(enc), B, P, E, ptr(out), stream())


def att_score_fwd(att_enc, dec_part, S, dec_slab, bias_da, wf, bf, B, P, A, e, att_dec_out=None):
    _cuda(att_enc, dec_part, bias_da, wf, bf, e, att_dec_out)
    call("capmi_att_score_fwd", ptr(att_enc), ptr(dec_part), S, dec_slab, ptr(bias_da), ptr(wf),
         ptr(bf), B, P, A, ptr(e), ptr(att_dec_out), stream())


def att_softmax_ctx_fwd(e, enc, B, P, E, bt, alpha_out, alpha_ld_b, awe_out, gate_part=None, S=0,
                        gate_slab=0, bias_fb=None, gate_out=None, x_out=None, ld_x=0):
    _cuda(e, enc, alpha_out, awe_out, gate_part, bias_fb, gate_out, x_out)
    call("capmi_att_softmax_ctx_fwd", ptr(e), ptr(enc), B, P, E, bt, ptr(alpha_out), alpha_ld_b,
         ptr(awe_out), ptr(gate_part), S, gate_slab, ptr(bias_fb), ptr(gate_out), ptr(x_out), ld_x,
         stream())


def lstm_cell_fwd(part, S, slab, xemb, hh_part, S2, slab2, c_prev, B, D, h_out, c_out, act_out):
    _cuda(part, xemb, hh_part, c_prev, h_out, c_out, act_out)
    call("capmi_lstm_cell_fwd", ptr(part), S, slab, ptr(xemb), ptr(hh_part), S2, slab2, ptr(c_prev), B,
         D, ptr(h_out), ptr(c_out), ptr(act_out), stream())


def dropout(inp, n, p, seed, out, seed_dev=None):
    """seed: host int; seed_dev: optional int64 device counter mixed into the seed (graphs)."""
    _cuda(inp, out)
    _cuda(seed_dev, dtype=torch.int64)
    call("capmi_dropout", ptr(inp), n, float(p), int(seed) & ((1 << 64) - 1), ptr(seed_dev), ptr(out),
         stream())


def counter_add(counter, v=1):
    _cuda(counter, dtype=torch.int64)
    call("capmi_counter_add", ptr(counter), int(v), stream())


def mask_rows_tb(x, bt_dev, T, B, cols, ld, r1=0, s2=0):
    _cuda(x)
    _cuda(bt_dev, dtype=torch.int32)
    call("capmi_mask_rows_tb", ptr(x), ptr(bt_dev), T, B, cols, ld, r1, s2, stream())


def ce_fwd_bwd(logits, caps, B, T, L, V, bt_dev, nrows, loss_rows, lse=None, dlogits=None,
               dl_time_major=False, gscale=None):
    _cuda(logits, loss_rows, lse, dlogits, gscale)
    _cuda(caps, dtype=torch.int64)
    _cuda(bt_dev, dtype=torch.int32)
    call("capmi_ce_fwd_bwd", ptr(logits), ptr(caps), B, T, L, V, ptr(bt_dev), nrows, ptr(loss_rows),
         ptr(lse), ptr(dlogits), int(dl_time_major), ptr(gscale), stream())


def alpha_reg_parts(B, P):
    return lib.capmi_alpha_reg_parts(B, P)


def alpha_reg(alphas, B, T, P, alpha_c, reg_part, dreg):
    """reg_part: alpha_reg_parts(B, P) floats whose sum is the regulariser value."""
    _cuda(alphas, reg_part, dreg)
    assert reg_part is None or reg_part.numel() >= alpha_reg_parts(B, P)
    call("capmi_alpha_reg", ptr(alphas), B, T, P, float(alpha_c), ptr(reg_part), ptr(dreg), stream())


def loss_finalize(loss_rows, n, nrows, reg_part, out):
    _cuda(loss_rows, reg_part, out)
    call("capmi_loss_finalize", ptr(loss_rows), n, nrows, ptr(reg_part),
         0 if reg_part is None else reg_part.numel(), ptr(out), stream())


def lstm_cell_bwd(dhd, dh_part, S, slab, dc_in, act, c_prev, c_cur, B, D, bt, dgates, dc_out):
    _cuda(dhd, dh_part, dc_in, act, c_prev, c_cur, dgates, dc_out)
    call("capmi_lstm_cell_bwd", ptr(dhd), ptr(dh_part), S, slab, ptr(dc_in), ptr(act), ptr(c_prev),
         ptr(c_cur), B, D, bt, ptr(dgates), ptr(dc_out), stream())


def att_alpha_expand(aq, rows, F, d, ap):
    """alphas over the F*F distinct rows -> over the reference's (F d)^2 positions (/ d^2)."""
    _cuda(aq, ap)
    assert aq.numel() >= rows * F * F and ap.numel() >= rows * (F * d) ** 2
    call("capmi_att_alpha_expand", ptr(aq), rows, F, d, ptr(ap), stream())


def att_dup_pick(inp, B, F, d, out):
    """out[b][qi][qj] = inp[b][qi*d][qj*d] (one representative per duplicated group)."""
    _cuda(inp, out)
    assert inp.numel() >= B * (F * d) ** 2 and out.numel() >= B * F * F
    call("capmi_att_dup_pick", ptr(inp), B, F, d, ptr(out), stream())


def att_ctx_bwd(part, S, slab, gate, awe, enc, B, P, E, dgp, dalpha, dawe_out=None):
    _cuda(part, gate, awe, enc, dgp, dalpha, dawe_out)
    call("capmi_att_ctx_bwd", ptr(part), S, slab, ptr(gate), ptr(awe), ptr(enc), B, P, E, ptr(dgp),
         ptr(dalpha), ptr(dawe_out), stream())


def att_enc_dinput(alpha, alpha_ld_b, dawe, dmean, B, T, P, E, denc):
    _cuda(alpha, dawe, dmean, denc)
    assert denc.numel() >= B * P * E and dawe.numel() >= T * B * E
    call("capmi_att_enc_dinput", ptr(alpha), alpha_ld_b, ptr(dawe), ptr(dmean), B, T, P, E, ptr(denc),
         stream())


def att_score_bwd(dalpha, dreg, dreg_ld_b, alpha, alpha_ld_b, att_enc, att_dec, wf, B, P, A, bt, de,
                  dad):
    _cuda(dalpha, dreg, alpha, att_enc, att_dec, wf, de, dad)
    call("capmi_att_score_bwd", ptr(dalpha), ptr(dreg), dreg_ld_b, ptr(alpha), alpha_ld_b, ptr(att_enc),
         ptr(att_dec), ptr(wf), B, P, A, bt, ptr(de), ptr(dad), stream())


def att_enc_grad(de, att_enc, att_dec, wf, T, B, P, A, datt_enc, wf_part, bf_part):
    _cuda(de, att_enc, att_dec, wf, datt_enc, wf_part, bf_part)
    n = ctypes.c_int(0)
    call("capmi_att_enc_grad", ptr(de), ptr(att_enc), ptr(att_dec), ptr(wf), T, B, P, A, ptr(datt_enc),
         ptr(wf_part), ptr(bf_part), ctypes.byref(n), stream())
    return n.value


def att_enc_grad_blocks(B, P):
    return ((P + 27) // 28) * B


# --------------------------------------------------------------------------------------
# fused recurrence kernels (decoder_step.hip)
# --------------------------------------------------------------------------------------
def dstep_gemm(segs, M, N, nt, S, epi, part, counters, gate_D=0):
    """segs: [(A, lda, W, ldw, K), ...] (1-3 K segments, fp32 views; A [M][K], W [N][K] row-major);
    epi: dict of capmi_dstep_epi fields (tensors or ints; ``mode`` one of CAPMI_DSTEP_*)."""
    arr = (DstepSeg * len(segs))()
    for i, (A, lda, W, ldw, K) in enumerate(segs):
        _cuda(A, W)
        arr[i].A, arr[i].lda, arr[i].W, arr[i].ldw, arr[i].K = ptr(A), int(lda), ptr(W), int(ldw), int(K)
    e = DstepEpi()
    for k, v in epi.items():
        if isinstance(v, torch.Tensor):
            _cuda(v)
            setattr(e, k, v.data_ptr())
        else:
            setattr(e, k, v)
    _cuda(part)
    _cuda(counters, dtype=torch.int32)
    call("capmi_dstep_gemm", arr, len(segs), int(M), int(N), int(nt), int(S), int(gate_D), ctypes.byref(e),
         ptr(part), part.numel(), ptr(counters), counters.numel(), stream())


def att_fwd_fused(att_enc, ad, S_a, slab_a, bias_da, ad_out, wf, bf, enc, gate, S_g, slab_g, bias_fb, gate_out,
                  B, P, A, E, bt, alpha_out, alpha_ld_b, awe_out, x_out, ld_x):
    _cuda(att_enc, ad, bias_da, ad_out, wf, bf, enc, gate, bias_fb, gate_out, alpha_out, awe_out, x_out)
    call("capmi_att_fwd_fused", ptr(att_enc), ptr(ad), S_a, slab_a, ptr(bias_da), ptr(ad_out), ptr(wf), ptr(bf),
         ptr(enc), ptr(gate), S_g, slab_g, ptr(bias_fb), ptr(gate_out), B, P, A, E, bt, ptr(alpha_out), alpha_ld_b,
         ptr(awe_out), ptr(x_out), ld_x, stream())


def att_bwd_fused(dx, S, slab, gate, awe, dgp, dawe_out, enc, alpha, alpha_ld_b, dreg, dreg_ld_b, att_enc, att_dec,
                  wf, B, P, A, E, bt, de, dad):
    _cuda(dx, gate, awe, dgp, dawe_out, enc, alpha, dreg, att_enc, att_dec, wf, de, dad)
    call("capmi_att_bwd_fused", ptr(dx), S, slab, ptr(gate), ptr(awe), ptr(dgp), ptr(dawe_out), ptr(enc), ptr(alpha),
         alpha_ld_b, ptr(dreg), dreg_ld_b, ptr(att_enc), ptr(att_dec), ptr(wf), B, P, A, E, bt, ptr(de), ptr(dad),
         stream())


# --------------------------------------------------------------------------------------
# optimiser
# --------------------------------------------------------------------------------------
def adam_clamp(p, g, m, v, lr, beta1, beta2, eps, bc1, bc2_sqrt, clip, step_dev=None):
    """step_dev: optional int64 device step counter (bias corrections computed on the device)."""
    _cuda(step_dev, dtype=torch.int64)
    name = "capmi_adam_clamp_f64" if p.dtype == torch.float64 else "capmi_adam_clamp"
    _cuda(p, g, m, v, dtype=p.dtype)
    call(name, ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(beta1), float(beta2),
         float(eps), float(bc1), float(bc2_sqrt), float(clip), ptr(step_dev), stream())


def embed_scatter_add(dx, ld_dx, caps, B, L, T, bt_dev, M, demb):
    _cuda(dx)
    _cuda(caps, dtype=torch.int64)
    _cuda(demb, dtype=None)
    call("capmi_embed_scatter_add", ptr(dx), ld_dx, ptr(caps), B, L, T, ptr(bt_dev), M, ptr(demb),
         int(demb.dtype == torch.float64), stream())


TILE_128, TILE_64, TILE_128x64, TILE_AUTO = CAPMI_TILE_128, CAPMI_TILE_64, CAPMI_TILE_128x64, CAPMI_TILE_AUTO
BNB_RELU_Y, BNB_RELU_OUT = 0, 1


# --------------------------------------------------------------------------------------
# timing events that can live inside HIP graphs (bench.py)
# --------------------------------------------------------------------------------------
class TimingEvent:
    """A HIP timing event; ``record()`` on the current stream becomes a graph node when that
    stream is being captured (torch refuses external events on ROCm)."""

    def __init__(self):
        h = ctypes.c_void_p()
        call("capmi_timing_event_create", ctypes.byref(h))
        self.h = h

    def record(self):
        call("capmi_timing_event_record", self.h, stream())

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        call("capmi_timing_elapsed_ms", self.h, end.h, ctypes.byref(ms))
        return float(ms.value)

    def __del__(self):
        try:
            lib.capmi_timing_event_destroy(self.h)
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def timed_launch(launch, start, stop):
    """Run ``launch`` (one capmi GEMM call, eager) with its kernel's dispatch start / end recorded
    into the TimingEvents ``start`` / ``stop`` (capmi_timing_arm: hipExtLaunchKernel, the AQL
    packet's own timestamps -- the duration rocprofv3 reports for that dispatch)."""
    call("capmi_timing_arm", start.h, stop.h)
    try:
        launch()
    finally:
        if lib.capmi_timing_disarm():
            raise CapmiError("timed_launch: the call launched no GEMM kernel")
