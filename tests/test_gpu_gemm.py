"""GPU: libcapmi GEMM / implicit-GEMM conv vs fp64 CPU references.

Tolerance: |C - C64| <= 4e-6 * (|A| |B|)_ij + 1e-6, i.e. a few fp32 roundings
of the row-by-column sum of magnitudes (the MFMA result is an exact fp32 fmaf
chain in a different k order than any CPU library)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _K():
    from capmi import kernels as K
    return K


def check(C, ref, ref_abs, what):
    err = (C.double().cpu() - ref).abs()
    tol = 4e-6 * ref_abs + 1e-6
    assert bool((err <= tol).all()), f"{what}: max err {float(err.max()):.3g}, worst ratio {float((err / tol).max()):.3g}"


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1


@pytest.mark.parametrize("tile", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,Kd", [(300, 200, 96), (64, 2048, 512), (129, 65, 52), (129, 65, 50), (1, 7, 3),
                                    (1000, 64, 300)])
def test_linear_fwd(tile, M, N, Kd):
    K = _K()
    X, W, b, b2 = rnd(M, Kd, seed=1), rnd(N, Kd, seed=2), rnd(N, seed=3), rnd(N, seed=4)
    C = torch.empty(M, N, device=DEV)
    K.gemm(K.problem(M, N, Kd, X.float().to(DEV), Kd, W.float().to(DEV), Kd, C, N,
                     bias=b.float().to(DEV), bias2=b2.float().to(DEV)), 0, 0, tile)
    ref = X @ W.T + b + b2
    check(C, ref, X.abs() @ W.abs().T + b.abs() + b2.abs(), "linear")


@pytest.mark.parametrize("tile", [0, 1, 2, 3])
@pytest.mark.parametrize("N,Kx", [(36, 44), (37, 45), (520, 260)])
def test_transposed_modes_and_remap(tile, N, Kx):
    """k-row operands (transposed staging in the v2 kernel; N % 4 != 0 takes the generic kernel)."""
    K = _K()
    # dW = dY^T X with dY stored batch-major (B,T,N) and read time-major through the 2-level remap
    B, T = 5, 7
    dY = rnd(B, T, N, seed=5)
    Xt = rnd(T * B, Kx, seed=6)  # time-major rows r = t*B + b
    C = torch.empty(N, Kx, device=DEV)
    K.gemm(K.problem(N, Kx, T * B, dY.float().to(DEV), T * N, Xt.float().to(DEV), Kx, C, Kx,
                     a_r1=B, a_s2=N), 1, 1, tile)
    dY_tm = dY.permute(1, 0, 2).reshape(T * B, N)
    check(C, dY_tm.T @ Xt, dY_tm.abs().T @ Xt.abs(), "MMAJOR x KROWS with remap")
    # dX = dY W (B operand row-major [K][N]) with output row remap to batch-major
    W = rnd(N, Kx, seed=7)
    out = torch.zeros(B, T, Kx, device=DEV)
    K.gemm(K.problem(T * B, Kx, N, dY.float().to(DEV), T * N, W.float().to(DEV), Kx, out, T * Kx,
                     a_r1=B, a_s2=N, c_r1=B, c_s2=Kx), 0, 1, tile)
    ref = (dY_tm @ W).view(T, B, Kx).permute(1, 0, 2)
    check(out, ref, (dY_tm.abs() @ W.abs()).view(T, B, Kx).permute(1, 0, 2), "KMAJOR x KROWS, C remap")


def test_splitk_grouped_and_reduce():
    K = _K()
    B, D, N1, N2 = 64, 512, 512, 2048
    h = rnd(B, D, seed=8)
    W1, W2 = rnd(N1, D, seed=9), rnd(N2, D, seed=10)
    s1, s2 = 4, 2
    P1 = torch.empty(s1, B, N1, device=DEV)
    P2 = torch.empty(s2, B, N2, device=DEV)
    hd = h.float().to(DEV)
    K.gemm([K.problem(B, N1, D, hd, D, W1.float().to(DEV), D, P1, N1, ksplit=s1, c_split_stride=B * N1),
            K.problem(B, N2, D, hd, D, W2.float().to(DEV), D, P2, N2, ksplit=s2, c_split_stride=B * N2)],
           0, 0, 1)
    out = torch.empty(B, N1, device=DEV)
    bias = rnd(N1, seed=11)
    K.splitk_reduce(P1, s1, B * N1, B, N1, N1, out, N1, bias=bias.float().to(DEV))
    check(out, h @ W1.T + bias, h.abs() @ W1.abs().T + bias.abs(), "split-K + reduce")
    check(P2.sum(0), h @ W2.T, h.abs() @ W2.abs().T, "grouped problem 2")


def test_colsum():
    K = _K()
    x = rnd(1000, 77, seed=12)
    out = torch.empty(77, device=DEV)
    work = torch.empty(K.colsum_work_size(1000, 77), device=DEV)
    K.colsum(x.float().to(DEV), 1000, 77, 77, out, work)
    check(out, x.sum(0), x.abs().sum(0), "colsum")


@pytest.mark.parametrize("tile", [0, 1, 2])
def test_bn_stats_epilogue(tile):
    K = _K()
    M, N, Kd = 1000, 96, 64
    X, W = rnd(M, Kd, seed=13), rnd(N, Kd, seed=14)
    C = torch.empty(M, N, device=DEV)
    tiles = K.stat_tiles(M)
    stats = torch.empty(tiles, N, 2, device=DEV)
    K.gemm(K.problem(M, N, Kd, X.float().to(DEV), Kd, W.float().to(DEV), Kd, C, N, stats=stats), 0, 0, tile)
    Cd = C.double().cpu()
    s = stats.double().cpu().sum(0)
    torch.testing.assert_close(s[:, 0], Cd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s[:, 1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("tile", [0, 3])
@pytest.mark.parametrize("k,stride,cin,cout,hw,prologue", [
    (3, 1, 64, 64, 14, True), (3, 2, 128, 128, 15, True), (1, 2, 64, 256, 14, False),
    (1, 1, 64, 256, 9, True), (3, 1, 48, 80, 7, True)])
def test_conv_nhwc(k, stride, cin, cout, hw, prologue, tile):
    K = _K()
    N = 3
    x = rnd(N, cin, hw, hw, seed=15)
    w = rnd(cout, cin, k, k, seed=16) * 0.1
    sc, sh = rnd(cin, seed=17), rnd(cin, seed=18)
    pad = k // 2
    xin = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)) if prologue else x
    ref = F.conv2d(xin, w, stride=stride, padding=pad)
    ref_abs = F.conv2d(xin.abs(), w.abs(), stride=stride, padding=pad)
    Ho = ref.shape[2]
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    wp = torch.empty(cout, k, k, cin, device=DEV)
    K.conv_weight_pack(w.float().to(DEV).contiguous(), wp)
    out = torch.empty(N * Ho * Ho, cout, device=DEV)
    geo = dict(N=N, H=hw, W=hw, Cin=cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
    K.gemm(K.problem(N * Ho * Ho, cout, k * k * cin, x_nhwc, 0, wp, k * k * cin, out, cout, conv=geo,
                     in_scale=sc.float().to(DEV) if prologue else None,
                     in_shift=sh.float().to(DEV) if prologue else None), 2, 0, tile)
    got = out.view(N, Ho, Ho, cout).permute(0, 3, 1, 2)
    check(got, ref, ref_abs, f"conv{k}x{k}/s{stride}")


def test_conv1_nchw_gather():
    K = _K()
    N, H = 2, 40
    x = rnd(N, 3, H, H, seed=19)
    w = rnd(64, 3, 7, 7, seed=20) * 0.1
    ref = F.conv2d(x, w, stride=2, padding=3)
    ref_abs = F.conv2d(x.abs(), w.abs(), stride=2, padding=3)
    Ho = ref.shape[2]
    out = torch.empty(N * Ho * Ho, 64, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=3, KH=7, KW=7, stride=2, pad=3, Ho=Ho, Wo=Ho)
    K.gemm(K.problem(N * Ho * Ho, 64, 147, x.float().to(DEV).contiguous(), 0, w.float().to(DEV).contiguous(),
                     147, out, 64, conv=geo), 3, 0, 0)
    check(out.view(N, Ho, Ho, 64).permute(0, 3, 1, 2), ref, ref_abs, "conv1 NCHW gather")


@pytest.mark.parametrize("tile", [1, 2, 3])
def test_conv1_nhwc4(tile):
    """conv1 as the encoder runs it: images -> NHWC4, weights packed with Cin padded to 4."""
    K = _K()
    N, H = 3, 46
    x = rnd(N, 3, H, H, seed=21)
    w = rnd(64, 3, 7, 7, seed=22) * 0.1
    ref = F.conv2d(x, w, stride=2, padding=3)
    ref_abs = F.conv2d(x.abs(), w.abs(), stride=2, padding=3)
    Ho = ref.shape[2]
    xd = x.float().to(DEV).contiguous()
    img4 = torch.full((N * H * H * 4,), float("nan"), device=DEV)
    K.image_nhwc4(xd, img4)
    assert torch.equal(img4.view(N, H, H, 4)[..., :3].cpu(), xd.permute(0, 2, 3, 1).cpu())
    assert float(img4.view(N, H, H, 4)[..., 3].abs().sum()) == 0.0
    wp = torch.full((64 * 49 * 4,), float("nan"), device=DEV)
    K.conv_weight_pack_pad(w.float().to(DEV).contiguous(), 4, wp)
    M = N * Ho * Ho
    out = torch.empty(M, 64, device=DEV)
    stats = torch.empty(K.stat_tiles(M), 64, 2, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=4, KH=7, KW=7, stride=2, pad=3, Ho=Ho, Wo=Ho)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, 64, 196, img4, 0, wp, 196, out, 64, conv=geo, stats=stats), 4, ws, tile)
    check(out.view(N, Ho, Ho, 64).permute(0, 3, 1, 2), ref, ref_abs, "conv1 NHWC4")
    s = stats.double().cpu().sum(0)
    torch.testing.assert_close(s[:, 0], out.double().cpu().sum(0), rtol=1e-5, atol=1e-3)


# ---------------------------------------------------------------------------------------
# stream-K (capmi_gemm_sk): persistent workgroups, k-prefixes parked in the workspace
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("M,N,Kd", [(64, 64, 4608), (1000, 96, 64), (3136, 256, 2304), (200, 130, 300),
                                    (12544, 64, 128)])
def test_gemm_sk_linear(tile, M, N, Kd):
    K = _K()
    X, W, b = rnd(M, Kd, seed=31), rnd(N, Kd, seed=32), rnd(N, seed=33)
    ws = K.gemm_workspace(DEV)
    C = torch.empty(M, N, device=DEV)
    stats = torch.empty(K.stat_tiles(M), N, 2, device=DEV)
    # the problem struct holds raw pointers: keep the device operands alive across both launches
    Xd, Wd, bd = X.float().to(DEV), W.float().to(DEV), b.float().to(DEV)
    prob = K.problem(M, N, Kd, Xd, Kd, Wd, Kd, C, N, bias=bd, stats=stats)
    K.gemm_sk(prob, 0, ws, tile)
    first = C.clone()
    K.gemm_sk(prob, 0, ws, tile)  # the workspace is reusable and the result deterministic
    torch.cuda.synchronize()
    assert torch.equal(first, C)
    nflags = torch.cuda.get_device_properties(0).multi_processor_count * 4 + 1
    assert int(ws[:nflags].abs().sum()) == 0, "stream-K flags not left zero (or spin timeout hit)"
    check(C, X @ W.T + b, X.abs() @ W.abs().T + b.abs(), "stream-K linear")
    Cd = C.double().cpu()
    s = stats.double().cpu().sum(0)
    torch.testing.assert_close(s[:, 0], Cd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s[:, 1], (Cd * Cd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("k,stride,cin,cout,hw", [(3, 1, 64, 128, 14), (3, 2, 128, 64, 15), (1, 1, 256, 64, 7)])
def test_conv_sk_prologue(k, stride, cin, cout, hw, tile=3):
    K = _K()
    N = 4
    x = rnd(N, cin, hw, hw, seed=34)
    w = rnd(cout, cin, k, k, seed=35) * 0.1
    sc, sh = rnd(cin, seed=36), rnd(cin, seed=37)
    pad = k // 2
    xin = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = F.conv2d(xin, w, stride=stride, padding=pad)
    ref_abs = F.conv2d(xin.abs(), w.abs(), stride=stride, padding=pad)
    Ho = ref.shape[2]
    x_nhwc = x.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    wp = torch.empty(cout, k, k, cin, device=DEV)
    K.conv_weight_pack(w.float().to(DEV).contiguous(), wp)
    M = N * Ho * Ho
    out = torch.empty(M, cout, device=DEV)
    stats = torch.empty(K.stat_tiles(M), cout, 2, device=DEV)
    geo = dict(N=N, H=hw, W=hw, Cin=cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, cout, k * k * cin, x_nhwc, 0, wp, k * k * cin, out, cout, conv=geo, stats=stats,
                        in_scale=sc.float().to(DEV), in_shift=sh.float().to(DEV)), 2, ws, tile)
    got = out.view(N, Ho, Ho, cout).permute(0, 3, 1, 2)
    check(got, ref, ref_abs, f"stream-K conv{k}x{k}/s{stride} tile {tile}")
    s = stats.double().cpu().sum(0)
    Cd = out.double().cpu()
    torch.testing.assert_close(s[:, 0], Cd.sum(0), rtol=1e-5, atol=1e-3)


def test_bn_finalize_shared_work():
    """BN finalize (one launch, last-arriving group finalizes) vs fp64, several widths sharing one
    zeroed work buffer, counters re-armed to zero after every call."""
    K = _K()
    work = torch.zeros(K.bn_work_doubles(2048), device=DEV, dtype=torch.float64)
    for it, (C, tiles) in enumerate([(64, 3136), (2048, 49), (256, 196), (64, 3136), (1024, 7), (512, 256), (128, 257)]):
        g = torch.Generator().manual_seed(40 + it)
        x = torch.randn(tiles * 64, C, generator=g, dtype=torch.float64) * 3 + 1
        rows = x.shape[0]
        stats = torch.stack([x.view(tiles, 64, C).sum(1), (x * x).view(tiles, 64, C).sum(1)], -1)
        gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
        rm, rv = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
        sd = [t.float().to(DEV) for t in (stats, gamma, beta, rm, rv)]
        scale, shift = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        K.bn_finalize(sd[0], tiles, C, rows, sd[1], sd[2], sd[3], sd[4], 0.1, 1e-5, scale, shift, work)
        torch.cuda.synchronize()
        mean, var = x.mean(0), x.var(0, unbiased=False)
        sc = gamma.double() / torch.sqrt(var + 1e-5)
        torch.testing.assert_close(scale.double().cpu(), sc, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(shift.double().cpu(), beta.double() - mean * sc, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(sd[3].double().cpu(), 0.9 * rm.double() + 0.1 * mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(sd[4].double().cpu(), 0.9 * rv.double() + 0.1 * x.var(0), rtol=1e-5, atol=1e-5)
        assert int(work[:64].view(torch.int32).abs().sum()) == 0, "arrival counters not re-armed"


@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("M,N,Kd", [(512, 2048, 784), (32, 2048, 588), (2048, 2560, 1536), (512, 64, 12544)])
def test_gemm_sk_transposed(tile, M, N, Kd):
    """dW = dY^T X (both operands stored as k rows) through stream-K: the decoder's weight grads."""
    K = _K()
    dY, X = rnd(Kd, M, seed=51), rnd(Kd, N, seed=52)
    dYd, Xd = dY.float().to(DEV), X.float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, N, Kd, dYd, M, Xd, N, C, N), 1, ws, tile, bmode=1)
    torch.cuda.synchronize()
    check(C, dY.T @ X, dY.abs().T @ X.abs(), "stream-K MMAJOR x KROWS")
    # and dX = dY W with W stored [k][n] (KMAJOR x KROWS)
    out = torch.empty(Kd, N, device=DEV)
    W = rnd(M, N, seed=53)
    Wd = W.float().to(DEV)
    K.gemm_sk(K.problem(Kd, N, M, dYd, M, Wd, N, out, N), 0, ws, tile, bmode=1)
    torch.cuda.synchronize()
    check(out, dY @ W, dY.abs() @ W.abs(), "stream-K KMAJOR x KROWS")


@pytest.mark.parametrize("k,stride,cin,cout,hw", [(3, 1, 256, 256, 14), (1, 1, 256, 1024, 14), (3, 2, 128, 128, 28),
                                                  (3, 1, 64, 192, 9)])
def test_conv_512_thread_tile(k, stride, cin, cout, hw):
    """CAPMI_TILE_128_W8 (128x128, 8 waves as 4x2, one workgroup per CU): the same conv contract,
    prologue and per-64-row-slice statistics (two wave rows per slice) as the 256-thread forms."""
    test_conv_sk_prologue(k, stride, cin, cout, hw, tile=4)


def test_dense_512_thread_tile():
    K = _K()
    M, N, Kd = 3000, 320, 640
    a, b = rnd(M, Kd, seed=61), rnd(N, Kd, seed=62)
    ad, bd = a.float().to(DEV), b.float().to(DEV)
    c = torch.empty(M, N, device=DEV)
    stats = torch.empty(K.stat_tiles(M), N, 2, device=DEV)
    ws = K.gemm_workspace(DEV)
    K.gemm_sk(K.problem(M, N, Kd, ad, Kd, bd, Kd, c, N, stats=stats), 0, ws, 4)
    torch.cuda.synchronize()
    check(c, a @ b.T, a.abs() @ b.abs().T, "512-thread dense")
    s = stats.double().cpu()
    Cd = c.double().cpu()
    for sl in range(K.stat_tiles(M)):
        rows = Cd[64 * sl: 64 * (sl + 1)]
        torch.testing.assert_close(s[sl, :, 0], rows.sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("cin,hw,cout,k,stride,want_nt", [(256, 14, 256, 3, 1, 512), (64, 56, 64, 3, 1, 256),
                                                          (128, 28, 512, 1, 1, 256), (512, 7, 2048, 1, 1, 512),
                                                          (64, 56, 256, 1, 1, 512)])
def test_auto_tile_picks_512_thread_form(cin, hw, cout, k, stride, want_nt):
    """TILE_AUTO's choice of workgroup form on encoder conv shapes (batch 64), as measured by
    tools/w8_ab.sh; with the bf16-operand flag the 256-thread kernel is always used."""
    K = _K()
    N = 64
    Ho = (hw + 2 * (k // 2) - k) // stride + 1
    M, Kd = N * Ho * Ho, k * k * cin
    x = torch.empty(N, hw, hw, cin, device=DEV)
    w = torch.empty(cout, Kd, device=DEV)
    y = torch.empty(M, cout, device=DEV)
    geo = dict(N=N, H=hw, W=hw, Cin=cin, KH=k, KW=k, stride=stride, pad=k // 2, Ho=Ho, Wo=Ho)
    sc = torch.empty(cin, device=DEV)
    prob = K.problem(M, cout, Kd, x, 0, w, Kd, y, cout, conv=geo, in_scale=sc, in_shift=sc)
    assert K.gemm_sk_plan(prob, 2, threads=True)[4] == want_nt
    assert K.gemm_sk_plan(prob, 2, bf16=True, threads=True)[4] == 256
    name = K.gemm_sk_kernel_name(prob, 2)
    assert name.startswith("gemm_nt8_kernel<2, true," if want_nt == 512 else "gemm_nt_kernel<")


@pytest.mark.parametrize("tile", [1, 2, 4])
def test_gemm_sk_hybrid_rounds(tile):
    """Grids of more than two rounds of tiles: the hybrid schedule runs all but the last 1-2
    rounds' worth of tiles whole (round-robin over the persistent workers) before stream-K
    balances the rest -- same result and statistics as the fp64 product, deterministic."""
    K = _K()
    M, N, Kd = 140000 if tile != 4 else 70000, 64 if tile != 4 else 256, 576
    X, W = rnd(M, Kd, seed=71), rnd(N, Kd, seed=72)
    Xd, Wd = X.float().to(DEV), W.float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    stats = torch.empty(K.stat_tiles(M), N, 2, device=DEV)
    ws = K.gemm_workspace(DEV)
    prob = K.problem(M, N, Kd, Xd, Kd, Wd, Kd, C, N, stats=stats)
    bm, bn, sk, _ = K.gemm_sk_plan(prob, 0, tile)
    slots = torch.cuda.get_device_properties(0).multi_processor_count * (4 if bm == bn == 64 else 2 if tile != 4 else 1)
    assert sk == 1 and ((M + bm - 1) // bm) * ((N + bn - 1) // bn) >= 2 * slots, "not a hybrid grid"
    K.gemm_sk(prob, 0, ws, tile)
    first = C.clone()
    K.gemm_sk(prob, 0, ws, tile)
    torch.cuda.synchronize()
    assert torch.equal(first, C)
    check(C, X @ W.T, X.abs() @ W.abs().T, f"hybrid stream-K tile {tile}")
    Cd = C.double().cpu()
    s = stats.double().cpu().sum(0)
    torch.testing.assert_close(s[:, 0], Cd.sum(0), rtol=1e-5, atol=1e-2)
