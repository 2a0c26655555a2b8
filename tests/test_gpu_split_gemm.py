"""GPU: split-staged dense GEMMs (capmi_gemm_ex / capmi_gemm_sk_ex with CAPMI_GEMM_SPLIT3 or
CAPMI_GEMM_BF16) in every layout the decoder uses, vs fp64 CPU references.

Tolerances (|C - C64| element-wise, S = (|A| |B|)_ij, the row-by-column sum of magnitudes):
  * SPLIT3 (fp32-accurate three-term split): 4e-6 * S + 1e-6, the fp32 MFMA kernel's bound
    (tests/test_gpu_gemm.py);
  * BF16 (operands rounded to bf16, RNE): 2^-7 * S + 1e-6 (two roundings of relative 2^-9 each,
    fp32 accumulation).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _K():
    from capmi import kernels as K
    return K


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1


def check(C, ref, ref_abs, flags, what):
    from capmi._lib import CAPMI_GEMM_SPLIT3
    err = (C.double().cpu() - ref).abs()
    tol = (4e-6 if flags == CAPMI_GEMM_SPLIT3 else 2.0 ** -7) * ref_abs + 1e-6
    assert bool((err <= tol).all()), f"{what}: max err {float(err.max()):.3g}, worst ratio {float((err / tol).max()):.3g}"


def _flags():
    from capmi._lib import CAPMI_GEMM_BF16, CAPMI_GEMM_SPLIT3
    return [CAPMI_GEMM_SPLIT3, CAPMI_GEMM_BF16]


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("tile", [0, 1, 2])
@pytest.mark.parametrize("M,N,Kd", [(300, 200, 96), (64, 2048, 512), (129, 65, 52), (1, 8, 4), (1536, 520, 36)])
def test_split_linear_fwd(fi, tile, M, N, Kd):
    K = _K()
    flags = _flags()[fi]
    X, W, b, b2 = rnd(M, Kd, seed=1), rnd(N, Kd, seed=2), rnd(N, seed=3), rnd(N, seed=4)
    C = torch.empty(M, N, device=DEV)
    K.gemm(K.problem(M, N, Kd, X.float().to(DEV), Kd, W.float().to(DEV), Kd, C, N,
                     bias=b.float().to(DEV), bias2=b2.float().to(DEV)), 0, 0, tile, flags=flags)
    ref = X @ W.T + b + b2
    check(C, ref, X.abs() @ W.abs().T + b.abs() + b2.abs(), flags, "A KMAJOR x W[N][K]")


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("tile", [0, 1, 2])
@pytest.mark.parametrize("N,Kx", [(36, 44), (520, 260), (8100, 512)])
def test_split_transposed_modes_and_remap(fi, tile, N, Kx):
    """k-row operands: the k-pair transposing store of the split staging."""
    K = _K()
    flags = _flags()[fi]
    B, T = 5, 7
    dY = rnd(B, T, N, seed=5)
    Xt = rnd(T * B, Kx, seed=6)
    # dW = dY^T X, dY batch-major read time-major through the 2-level row remap (MMAJOR x KROWS)
    C = torch.empty(N, Kx, device=DEV)
    K.gemm(K.problem(N, Kx, T * B, dY.float().to(DEV), T * N, Xt.float().to(DEV), Kx, C, Kx,
                     a_r1=B, a_s2=N), 1, 1, tile, flags=flags)
    dY_tm = dY.permute(1, 0, 2).reshape(T * B, N)
    check(C, dY_tm.T @ Xt, dY_tm.abs().T @ Xt.abs(), flags, "MMAJOR x KROWS with remap")
    # dX = dY W (KMAJOR x KROWS) with output row remap, beta = 1 accumulation
    W = rnd(N, Kx, seed=7)
    C0 = rnd(B, T, Kx, seed=8)
    out = C0.float().to(DEV)
    K.gemm(K.problem(T * B, Kx, N, dY.float().to(DEV), T * N, W.float().to(DEV), Kx, out, T * Kx,
                     a_r1=B, a_s2=N, c_r1=B, c_s2=Kx, beta=1.0), 0, 1, tile, flags=flags)
    ref = (dY_tm @ W).view(T, B, Kx).permute(1, 0, 2) + C0
    ref_abs = (dY_tm.abs() @ W.abs()).view(T, B, Kx).permute(1, 0, 2) + C0.abs()
    check(out, ref, ref_abs, flags, "KMAJOR x KROWS, C remap, beta 1")


@pytest.mark.parametrize("fi", [0, 1])
def test_split_grouped_ksplit(fi):
    """The decoder's per-timestep form: grouped problems sharing A, k-split partial slabs."""
    K = _K()
    flags = _flags()[fi]
    B, D, N1, N2 = 64, 512, 512, 2048
    h = rnd(B, D, seed=8)
    W1, W2 = rnd(N1, D, seed=9), rnd(N2, D, seed=10)
    s1, s2 = 4, 2
    P1 = torch.empty(s1, B, N1, device=DEV)
    P2 = torch.empty(s2, B, N2, device=DEV)
    hd = h.float().to(DEV)
    K.gemm([K.problem(B, N1, D, hd, D, W1.float().to(DEV), D, P1, N1, ksplit=s1, c_split_stride=B * N1),
            K.problem(B, N2, D, hd, D, W2.float().to(DEV), D, P2, N2, ksplit=s2, c_split_stride=B * N2)],
           0, 0, 1, flags=flags)
    check(P1.sum(0), h @ W1.T, h.abs() @ W1.abs().T, flags, "grouped 1")
    check(P2.sum(0), h @ W2.T, h.abs() @ W2.abs().T, flags, "grouped 2")
    # backward form: dh = dG W (KROWS), grouped with k-split
    dG = rnd(B, 4 * D, seed=11)
    Whh = rnd(4 * D, D, seed=12)
    s = 4
    P = torch.empty(s, B, D, device=DEV)
    K.gemm([K.problem(B, D, 4 * D, dG.float().to(DEV), 4 * D, Whh.float().to(DEV), D, P, D, ksplit=s,
                      c_split_stride=B * D)], 0, 1, 1, flags=flags)
    check(P.sum(0), dG @ Whh, dG.abs() @ Whh.abs(), flags, "KROWS k-split")


@pytest.mark.parametrize("fi", [0, 1])
@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("mode,M,N,Kd", [((0, 0), 1536, 8100, 512), ((0, 1), 1536, 512, 8100),
                                          ((1, 1), 8100, 512, 1536), ((1, 1), 2048, 2048, 3136),
                                          ((0, 0), 100, 64, 4096)])
def test_split_stream_k(fi, tile, mode, M, N, Kd):
    """capmi_gemm_sk_ex with the split flags (stream-K / hybrid grids of the hoisted GEMMs)."""
    K = _K()
    flags = _flags()[fi]
    am, bm = mode
    A = rnd(Kd, M, seed=13) if am == 1 else rnd(M, Kd, seed=13)
    Bm = rnd(Kd, N, seed=14) if bm == 1 else rnd(N, Kd, seed=14)
    C = torch.empty(M, N, device=DEV)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, N, Kd, A.float().to(DEV), M if am == 1 else Kd, Bm.float().to(DEV),
                        N if bm == 1 else Kd, C, N), am, ws, tile, bm, flags=flags)
    Am = A.T if am == 1 else A
    Bk = Bm if bm == 1 else Bm.T
    check(C, Am @ Bk, Am.abs() @ Bk.abs(), flags, f"stream-K mode {mode}")
    torch.cuda.synchronize()
    K.sk_check([ws])


def test_split3_error_not_above_fp32_kernel():
    """Relative L2 error of SPLIT3 vs fp64 is at most 2x the fp32 MFMA kernel's on the same problem."""
    K = _K()
    from capmi._lib import CAPMI_GEMM_SPLIT3
    M, N, Kd = 1536, 8100, 512
    X, W = rnd(M, Kd, seed=15), rnd(N, Kd, seed=16)
    ref = X @ W.T
    errs = []
    for flags in (0, CAPMI_GEMM_SPLIT3):
        C = torch.empty(M, N, device=DEV)
        K.gemm(K.problem(M, N, Kd, X.float().to(DEV), Kd, W.float().to(DEV), Kd, C, N), 0, 0, 1, flags=flags)
        errs.append(float((C.double().cpu() - ref).norm() / ref.norm()))
    assert errs[1] <= 2 * errs[0] + 1e-9, errs


@pytest.mark.parametrize("tile", [1, 2, 3])
def test_split3_conv1_nhwc4_stats(tile):
    """conv1 as the x3 encoder runs it (CAPMI_GEMM_SPLIT3 on the NHWC4 images, K = 196) with the BN
    statistics epilogue: fp32 tolerance vs fp64, statistics = sums of the stored output."""
    import torch.nn.functional as F
    from capmi._lib import CAPMI_GEMM_SPLIT3
    K = _K()
    N, H = 3, 46
    x = rnd(N, 3, H, H, seed=21)
    w = rnd(64, 3, 7, 7, seed=22) * 0.1
    ref = F.conv2d(x, w, stride=2, padding=3)
    ref_abs = F.conv2d(x.abs(), w.abs(), stride=2, padding=3)
    Ho = ref.shape[2]
    img4 = torch.empty(N * H * H * 4, device=DEV)
    K.image_nhwc4(x.float().to(DEV).contiguous(), img4)
    wp = torch.empty(64 * 49 * 4, device=DEV)
    K.conv_weight_pack_pad(w.float().to(DEV).contiguous(), 4, wp)
    M = N * Ho * Ho
    out = torch.empty(M, 64, device=DEV)
    stats = torch.empty(K.stat_tiles(M), 64, 2, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=4, KH=7, KW=7, stride=2, pad=3, Ho=Ho, Wo=Ho)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, 64, 196, img4, 0, wp, 196, out, 64, conv=geo, stats=stats), 4, ws, tile,
              flags=CAPMI_GEMM_SPLIT3)
    check(out.view(N, Ho, Ho, 64).permute(0, 3, 1, 2), ref, ref_abs, CAPMI_GEMM_SPLIT3, "conv1 NHWC4 x3")
    s = stats.double().cpu().sum(0)
    torch.testing.assert_close(s[:, 0], out.double().cpu().sum(0), rtol=1e-5, atol=1e-3)
    assert "gemm_nts_kernel" in K.gemm_sk_kernel_name(
        K.problem(M, 64, 196, img4, 0, wp, 196, out, 64, conv=geo, stats=stats), 4, tile=tile, flags=CAPMI_GEMM_SPLIT3)


@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("k,stride,cin,cout,hw", [(3, 1, 64, 64, 14), (3, 2, 128, 128, 15), (1, 1, 64, 256, 9)])
def test_split3_conv_nhwc(k, stride, cin, cout, hw, tile):
    """The conv mode without prologue (the fine-tune data gradients' form) under CAPMI_GEMM_SPLIT3."""
    import torch.nn.functional as F
    from capmi._lib import CAPMI_GEMM_SPLIT3
    K = _K()
    N = 3
    x = rnd(N, cin, hw, hw, seed=15)
    w = rnd(cout, cin, k, k, seed=16) * 0.1
    pad = k // 2
    ref = F.conv2d(x, w, stride=stride, padding=pad)
    ref_abs = F.conv2d(x.abs(), w.abs(), stride=stride, padding=pad)
    Ho = ref.shape[2]
    wp = torch.empty(cout, k, k, cin, device=DEV)
    K.conv_weight_pack(w.float().to(DEV).contiguous(), wp)
    out = torch.empty(N * Ho * Ho, cout, device=DEV)
    geo = dict(N=N, H=hw, W=hw, Cin=cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(N * Ho * Ho, cout, k * k * cin, x.permute(0, 2, 3, 1).contiguous().float().to(DEV), 0,
                        wp, k * k * cin, out, cout, conv=geo), 2, ws, tile, flags=CAPMI_GEMM_SPLIT3)
    check(out.view(N, Ho, Ho, cout).permute(0, 3, 1, 2), ref, ref_abs, CAPMI_GEMM_SPLIT3, f"conv{k} x3")
