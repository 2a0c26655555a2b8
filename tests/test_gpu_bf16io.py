"""GPU: the bf16-activation conv path (CAPMI_GEMM_BF16_IO, gemm_bf16.hip) and its elementwise
kernels, for BASELINE config 5 (bf16). Operands are bf16 in HBM, products are exact in fp32 and
accumulate in fp32, and the output is rounded to bf16 once (RNE). So against the fp64 product of
the same bf16 operands, every output element must equal round_bf16(ref) up to one bf16 ulp (the
fp32 accumulation may land on the other side of a rounding boundary): |out - ref| <= 2^-7 |ref| +
2^-20 sum_k |a_k b_k| element-wise, and relative L2 <= 4e-3. BN statistics are the fp32 sums of the STORED values:
checked against torch sums of the bf16 output (rtol 1e-5)."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * scale).to(BF)


def _check_out(out, ref, mag):
    """mag = sum_k |a_k b_k| per element: the fp32 accumulation error allowance (2^-20 mag) on top
    of one bf16 ulp (<= 2^-7 |x|); it matters only where the sum cancels to far below its terms."""
    o = out.double().cpu()
    bad = int(((o - ref).abs() > ref.abs() * 2.0 ** -7 + mag * 2.0 ** -20 + 1e-30).sum())
    assert bad == 0, (bad, float((o - ref).abs().max()))
    assert rel_err(o, ref) < 4e-3, rel_err(o, ref)


def _check_stats(stats, out, rows, C):
    from capmi import kernels as K
    tiles = K.stat_tiles(rows)
    st = stats[: tiles * C * 2].view(tiles, C, 2).double().cpu().sum(0)
    o = out.reshape(rows, C).double().cpu()
    torch.testing.assert_close(st[:, 0], o.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(st[:, 1], (o * o).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,tile", [
    (64, 14, 256, 256, 3, 1, 3),   # layer3 conv2 at batch 64: 196 tiles, the four-deep DMA ring on 512 threads
    (2, 14, 256, 256, 3, 1, 3),    # small grid
    (2, 56, 64, 64, 3, 1, 3),      # layer1 conv2: N = 64 -> 128x64
    (12, 56, 64, 64, 3, 1, 3),     # 294 tiles of 128x64: the two-deep DMA ring on 256 threads
    (48, 28, 64, 128, 3, 1, 3),    # 294 tiles of 128x128: the two-deep DMA ring on 512 threads
    (1, 28, 128, 128, 3, 2, 3),    # stride-2 3x3 (first block of layer3), M % 128 != 0
    (2, 14, 128, 256, 1, 2, 3),    # stride-2 1x1 downsample
    (3, 7, 512, 192, 1, 1, 2),     # forced 128x64, N not a multiple of 64
])
def test_bf16io_conv(N, H, Cin, Cout, k, s, tile):
    from capmi import kernels as K
    from capmi._lib import CAPMI_A_CONV_NHWC
    pad = k // 2
    Ho = (H + 2 * pad - k) // s + 1
    x = _rand((N, H, H, Cin), 1, 2.0)
    w = _rand((Cout, k, k, Cin), 2, 0.1)
    conv = lambda u, v: F.conv2d(u.permute(0, 3, 1, 2), v.permute(0, 3, 1, 2), stride=s,  # noqa: E731
                                 padding=pad).permute(0, 2, 3, 1)
    ref, mag = conv(x.double(), w.double()), conv(x.double().abs(), w.double().abs())
    rows = N * Ho * Ho
    out = torch.full((N, Ho, Ho, Cout), float("nan"), device=DEV, dtype=BF)
    stats = torch.empty(K.stat_tiles(rows) * Cout * 2, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=s, pad=pad, Ho=Ho, Wo=Ho)
    xd, wd = x.to(DEV), w.to(DEV).contiguous()  # kept alive: the problem holds raw pointers
    prob = K.problem_bf16(rows, Cout, k * k * Cin, xd, 0, wd, k * k * Cin, out, Cout, stats=stats, conv=geo)
    ws = K.gemm_workspace(DEV)
    K.gemm_bf16(prob, CAPMI_A_CONV_NHWC, ws, tile)
    torch.cuda.synchronize()
    _check_out(out, ref, mag)
    _check_stats(stats, out, rows, Cout)
    # stream-K leaves its workspace reusable: a second launch is bit-identical
    out2 = torch.empty_like(out)
    prob2 = K.problem_bf16(rows, Cout, k * k * Cin, xd, 0, wd, k * k * Cin, out2, Cout, stats=stats, conv=geo)
    K.gemm_bf16(prob2, CAPMI_A_CONV_NHWC, ws, tile)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), out2.view(torch.int16))


# K <= 256 under AUTO: the one-stage 128x64 form (round 5) -- the l3 c3 shape, a partial last row tile, N not a
# multiple of 64 (general epilogue), layer1's K = 64; K = 512 / 576 / 1024: the DMA ring
@pytest.mark.parametrize("M,N,Kd,tile", [(12544, 256, 1024, 3), (1000, 512, 256, 3), (300, 64, 128, 3),
                                         (12544, 1024, 256, 3), (500, 200, 192, 3), (2000, 256, 64, 3),
                                         (40000, 128, 512, 3), (3000, 320, 576, 3)])
def test_bf16io_dense(M, N, Kd, tile):
    from capmi import kernels as K
    from capmi._lib import CAPMI_A_KMAJOR
    a, b = _rand((M, Kd), 5), _rand((N, Kd), 6)
    ref, mag = a.double() @ b.double().T, a.double().abs() @ b.double().abs().T
    c = torch.empty(M, N, device=DEV, dtype=BF)
    stats = torch.empty(K.stat_tiles(M) * N * 2, device=DEV)
    ad, bd, ws = a.to(DEV), b.to(DEV), K.gemm_workspace(DEV)  # kept alive: raw pointers in the problem
    prob = K.problem_bf16(M, N, Kd, ad, Kd, bd, Kd, c, N, stats=stats)
    K.gemm_bf16(prob, CAPMI_A_KMAJOR, ws, tile)
    torch.cuda.synchronize()
    _check_out(c, ref, mag)
    _check_stats(stats, c, M, N)


def test_bf16io_rejects_unsupported():
    from capmi import kernels as K
    from capmi._lib import CAPMI_A_CONV_NHWC, CapmiError
    x = _rand((1, 8, 8, 32), 1).to(DEV)  # Cin % 64 != 0
    w = _rand((64, 3, 3, 32), 2).to(DEV)
    out = torch.empty(1, 8, 8, 64, device=DEV, dtype=BF)
    geo = dict(N=1, H=8, W=8, Cin=32, KH=3, KW=3, stride=1, pad=1, Ho=8, Wo=8)
    with pytest.raises(CapmiError):
        K.gemm_bf16(K.problem_bf16(64, 64, 288, x, 0, w, 288, out, 64, conv=geo), CAPMI_A_CONV_NHWC,
                    K.gemm_workspace(DEV))


def test_bf16_elementwise():
    from capmi import kernels as K
    rows, C = 1000, 256
    y, r = _rand((rows, C), 7, 3.0), _rand((rows, C), 8, 3.0)
    g = torch.Generator().manual_seed(9)
    s, b = torch.rand(C, generator=g) + 0.5, torch.rand(C, generator=g) - 0.5
    rs, rb = torch.rand(C, generator=g) + 0.5, torch.rand(C, generator=g) - 0.5
    yd, rd = y.to(DEV), r.to(DEV)
    sd, bd, rsd, rbd = (v.to(DEV) for v in (s, b, rs, rb))
    # x = relu(fmaf(y, s, b)) rounded to bf16 once
    x = torch.empty(rows, C, device=DEV, dtype=BF)
    K.bn_relu_bf16(yd, sd, bd, rows, C, x)
    want = torch.relu((y.double() * s.double() + b.double()).float()).to(BF)  # fmaf, then RNE
    assert torch.equal(x.cpu().view(torch.int16), want.view(torch.int16))
    # tail, identity and downsample residual
    out = torch.empty(rows, C, device=DEV, dtype=BF)
    K.bn_add_relu_bf16(yd, sd, bd, rd, out, rows, C)
    want = torch.relu(torch.addcmul(b, y.float(), s) + r.float()).to(BF)
    assert (out.cpu().float() - want.float()).abs().max() <= 2 ** -7 * want.float().abs().max()
    K.bn_add_relu_bf16(yd, sd, bd, rd, out, rows, C, res_scale=rsd, res_shift=rbd)
    want = torch.relu(torch.addcmul(b, y.float(), s) + torch.addcmul(rb, r.float(), rs)).to(BF)
    assert (out.cpu().float() - want.float()).abs().max() <= 2 ** -7 * want.float().abs().max()
    # fp32 -> bf16 is torch's RNE cast bit for bit
    f = torch.randn(4096, generator=g) * 100
    h = torch.empty(4096, device=DEV, dtype=BF)
    K.f32_to_bf16(f.to(DEV), h)
    assert torch.equal(h.cpu().view(torch.int16), f.to(BF).view(torch.int16))
    # adaptive average pool 7x7 -> 14x14 (the encoder's replicate) and 9x9 -> 4x4
    for Hh, O in ((7, 14), (9, 4)):
        m = _rand((2, Hh, Hh, 64), 10)
        o = torch.empty(2, O, O, 64, device=DEV)
        K.adaptive_avgpool_bf16(m.to(DEV), 2, Hh, Hh, 64, O, O, o)
        want = F.adaptive_avg_pool2d(m.float().permute(0, 3, 1, 2), (O, O)).permute(0, 2, 3, 1)
        torch.testing.assert_close(o.cpu(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("H,Cin,Cout,k,s,name", [
    (7, 512, 512, 3, 1, "gemm_bf16_kernel<128, 64, 2, false, 4>"),    # layer4 3x3: 100 tiles of 128x128, K = 4608
    (14, 512, 512, 3, 2, "gemm_bf16_kernel<128, 64, 2, false, 4>"),   # layer4.0's stride-2 3x3
    (7, 2048, 512, 1, 1, "gemm_bf16_kernel<128, 64, 0, false, 4>"),   # layer4 c1 (K = 2048, dense rows)
])
def test_bf16io_layer4_exact_shapes(H, Cin, Cout, k, s, name):
    """layer4's convs at batch 64 run 128x64 tiles on grids of 128x128 tiles that fill at most half
    the CUs (round 5), since round 6 on the four-deep DMA ring (gemm.hip bf16_io_plan) -- checked element-wise at their
    exact shapes, the instantiation asserted through the launcher's own plan. fp64 reference on the device (im2col +
    GEMM)."""
    from capmi import kernels as K
    from capmi._lib import CAPMI_A_CONV_NHWC, CAPMI_A_KMAJOR
    N, pad = 64, k // 2
    Ho = (H + 2 * pad - k) // s + 1
    x = _rand((N, H, H, Cin), 31, 2.0).to(DEV)
    w = _rand((Cout, k, k, Cin), 32, 0.05).to(DEV).contiguous()
    rows, Kd = N * Ho * Ho, k * k * Cin
    out = torch.full((N, Ho, Ho, Cout), float("nan"), device=DEV, dtype=BF)
    stats = torch.empty(K.stat_tiles(rows) * Cout * 2, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=s, pad=pad, Ho=Ho, Wo=Ho)
    if k == 1 and s == 1:  # the runner's 1x1 form: dense rows (capmi.resnet.EncoderRunner._conv_bf16)
        prob, mode = K.problem_bf16(rows, Cout, Kd, x, Cin, w, Kd, out, Cout, stats=stats), CAPMI_A_KMAJOR
    else:
        prob, mode = K.problem_bf16(rows, Cout, Kd, x, 0, w, Kd, out, Cout, stats=stats, conv=geo), CAPMI_A_CONV_NHWC
    assert K.gemm_bf16_kernel_name(prob, mode) == name
    K.gemm_bf16(prob, mode, K.gemm_workspace(DEV), K.TILE_AUTO)
    torch.cuda.synchronize()
    assert K.last_launch_name() == name

    def im2col_gemm(u, v):  # (N, H, H, Cin) x (Cout, k, k, Cin) -> (rows, Cout), fp64 on the device
        cols = F.unfold(u.permute(0, 3, 1, 2), k, padding=pad, stride=s)            # (N, Cin k k, Ho Wo)
        wm = v.permute(0, 3, 1, 2).reshape(Cout, Kd)                                 # (ci, kh, kw) order
        return (wm @ cols).permute(0, 2, 1).reshape(rows, Cout)
    ref = im2col_gemm(x.double(), w.double()).cpu()
    mag = im2col_gemm(x.double().abs(), w.double().abs()).cpu()
    _check_out(out.reshape(rows, Cout), ref, mag)
    _check_stats(stats, out, rows, Cout)
