"""GPU: the fp32-accurate three-term bf16 split GEMM (CAPMI_GEMM_X3, csrc/gemm_x3.hip).

The split a = a0 + a1 + a2 (bf16 terms) is exact; the GEMM keeps the six cross products above
2^-23 |a||b| and accumulates in fp32. Tolerance: the fp32 kernel's (tests/test_gpu_gemm.py),
|C - C64| <= 4e-6 (|A||B|)_ij + 1e-6 element-wise against the fp64 product of the same fp32
operands; and the relative L2 error may not exceed 2x the native fp32 MFMA kernel's on the same
problem (it is measured, not assumed, to be of the same size)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    from capmi import kernels as K
    return K


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1).float()


def split3(w):
    K = _K()
    out = torch.empty(3 * w.numel(), device=DEV, dtype=torch.bfloat16)
    K.split3_bf16(w.contiguous(), out)
    return out


def _errs(C, ref, ref_abs):
    err = (C.double().cpu() - ref).abs()
    tol = 4e-6 * ref_abs + 1e-6
    return float((err / tol).max()), float((C.double().cpu() - ref).norm() / ref.norm())


def test_split3_exact():
    """in = h0 + h1 + h2 exactly (fp64 sum of the bf16 terms), over a wide exponent range."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(1 << 16, generator=g) * torch.exp2(torch.randint(-60, 60, (1 << 16,), generator=g).float()))
    # exact for |x| below the bf16 maximum (3.39e38) and above 2^-110 (below it the low terms
    # fall into the subnormal range: an absolute error under 2^-126, far beneath any activation)
    x[:8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 1e30, -3e-30, 1.0000001, 0.33333334])
    h = split3(x.to(DEV)).cpu().view(3, -1).double()
    assert torch.equal(h.sum(0), x.double())
    assert bool((h[1].abs() <= h[0].abs() * 2 ** -8).all()) and bool((h[2].abs() <= h[0].abs() * 2 ** -16).all())


@pytest.mark.parametrize("M,N,Kd,tile", [(300, 200, 96, 3), (12544, 512, 2048, 3), (1536, 8100, 512, 3),
                                         (129, 64, 64, 3), (1, 7, 32, 3), (4096, 1024, 256, 2), (700, 128, 4608, 3)])
def test_x3_dense(M, N, Kd, tile):
    K = _K()
    X, W, b = rnd(M, Kd, seed=1), rnd(N, Kd, seed=2), rnd(N, seed=3)
    Xd, Wd = X.to(DEV), W.to(DEV)
    ws = K.gemm_workspace(DEV)
    C = torch.full((M, N), float("nan"), device=DEV)
    K.gemm_x3(K.problem(M, N, Kd, Xd, Kd, split3(Wd), Kd, C, N, bias=b.to(DEV)), 0, ws, tile)
    Cn = torch.empty(M, N, device=DEV)
    K.gemm_sk(K.problem(M, N, Kd, Xd, Kd, Wd, Kd, Cn, N, bias=b.to(DEV)), 0, ws)
    torch.cuda.synchronize()
    K.sk_check([ws])
    ref = X.double() @ W.double().T + b.double()
    ref_abs = X.double().abs() @ W.double().abs().T + b.double().abs()
    r3, e3 = _errs(C, ref, ref_abs)
    rn, en = _errs(Cn, ref, ref_abs)
    assert r3 <= 1.0, (r3, e3, rn, en)
    assert e3 <= 2 * en + 1e-9, (e3, en)


@pytest.mark.parametrize("N,H,Cin,Cout,k,stride,pro", [
    (4, 14, 256, 256, 3, 1, True), (4, 28, 128, 128, 3, 2, True), (2, 56, 64, 64, 3, 1, True),
    (3, 14, 1024, 256, 1, 1, False), (2, 28, 256, 512, 1, 2, False), (2, 7, 512, 2048, 1, 1, True),
    (64, 14, 256, 256, 3, 1, True)])
def test_x3_conv_prologue_stats(N, H, Cin, Cout, k, stride, pro):
    """Implicit-GEMM conv on NHWC with the BN-apply + ReLU prologue (input relu(x*s+b), padding
    zeros AFTER it) and the per-64-row-slice BN statistics of the stored output."""
    K = _K()
    pad = k // 2
    Ho = (H + 2 * pad - k) // stride + 1
    x = rnd(N, H, H, Cin, seed=4)
    w = rnd(Cout, k, k, Cin, seed=5) * (2.0 / (k * k * Cin)) ** 0.5
    s, b = rnd(Cin, seed=6) + 1.0, rnd(Cin, seed=7)
    xin = torch.relu(x * s + b) if pro else x
    rows = N * Ho * Ho
    Kd = k * k * Cin
    ws = K.gemm_workspace(DEV)
    stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=DEV)
    out = torch.empty(rows, Cout, device=DEV)
    geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
    wd = w.reshape(Cout, Kd).to(DEV)
    # operands held until the launch has run: the problem keeps raw pointers only
    xd, w3, sd, bd = x.to(DEV), split3(wd), s.to(DEV), b.to(DEV)
    prob = K.problem(rows, Cout, Kd, xd, 0, w3, Kd, out, Cout, conv=geo, stats=stats,
                     in_scale=sd if pro else None, in_shift=bd if pro else None)
    K.gemm_x3(prob, 2, ws)
    torch.cuda.synchronize()
    K.sk_check([ws])
    xi = xin.double().permute(0, 3, 1, 2)
    wt = w.double().permute(0, 3, 1, 2)
    ref = F.conv2d(xi, wt, stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    ref_abs = F.conv2d(xi.abs(), wt.abs(), stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    r3, _ = _errs(out, ref, ref_abs)
    assert r3 <= 1.0, r3
    o = out.double().cpu()
    st = stats.double().cpu()[: 2 * ((rows + 63) // 64) * Cout].view(-1, Cout, 2)
    torch.testing.assert_close(st[..., 0].sum(0), o.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(st[..., 1].sum(0), (o * o).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("B,H", [(2, 224), (64, 224)])
def test_encoder_x3_matches_oracle(B, H):
    """The whole train-mode encoder with every eligible conv on the x3 GEMM: within 2x the fp32 CPU
    path's own error against fp64 (the rule of tests/test_gpu_encoder.py)."""
    import os
    import gen
    from helpers import rel_err, t
    from models.encoder import EncoderAttention
    from oracle.resnet_ref import build_resnet101, encoder_attention_forward
    names = ["conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4"]
    env = os.environ.get("OMP_NUM_THREADS", "")
    torch.set_num_threads(int(env) if env.isdigit() and int(env) > 0 else 8)
    seed = 77
    params = gen.resnet101_params(seed)
    enc = EncoderAttention()
    sd = enc.state_dict()
    for k_, v in params.items():
        head, rest = k_.split(".", 1)
        sd[f"resnet.{names.index(head)}.{rest}"] = t(v).clone()
    enc.load_state_dict(sd)
    enc = enc.to(DEV).train()
    enc.set_compute_precision("fp32-x3")
    x = gen.images(seed, B, H, H)
    with torch.no_grad():
        y = enc(t(x, DEV)).cpu()
    r32, r64 = build_resnet101(params).train(), build_resnet101(params).double().train()
    with torch.no_grad():
        y32 = encoder_attention_forward(r32, t(x))
        y64 = encoder_attention_forward(r64, t(x).double())
    e_gpu, e_cpu = rel_err(y, y64), rel_err(y32, y64)
    assert e_gpu <= 2 * e_cpu + 1e-6, (e_gpu, e_cpu)


@pytest.mark.parametrize("rows,C", [(1000, 96), (12544, 256), (3137, 1024), (5, 12), (777, 2048)])
def test_bn_relu_split3_exact(rows, C):
    """The split planes of relu(y*s+b) sum exactly (fp64) to the fp32 value torch computes (any C: the
    grid keeps one channel group per thread)."""
    K = _K()
    y, s, b = rnd(rows, C, seed=8) * 3, rnd(C, seed=9) + 1.5, rnd(C, seed=10)
    out = torch.empty(3 * rows * C, device=DEV, dtype=torch.bfloat16)
    K.bn_relu_split3(y.to(DEV), s.to(DEV), b.to(DEV), rows, C, out)
    torch.cuda.synchronize()
    h = out.cpu().view(3, rows, C).double()
    want = torch.relu(torch.addcmul(b, y, s))  # fma order: y*s + b, rounded once (as fmaf)
    assert torch.equal(h.sum(0), want.double()) or float((h.sum(0) - want.double()).abs().max()) <= \
        float(want.abs().max()) * 2 ** -23
    out2 = torch.empty(3 * rows * C, device=DEV, dtype=torch.bfloat16)
    K.bn_relu_split3(y.to(DEV), None, None, rows, C, out2)
    torch.cuda.synchronize()
    assert torch.equal(out2.cpu().view(3, rows, C).double().sum(0), y.double())


@pytest.mark.parametrize("N,H,Cin,Cout,k,stride,pro", [
    (4, 14, 256, 256, 3, 1, True), (4, 28, 128, 128, 3, 2, True), (2, 56, 64, 256, 1, 1, True),
    (3, 14, 256, 1024, 1, 1, True), (2, 7, 512, 2048, 1, 1, False), (64, 14, 256, 256, 3, 1, True),
    (1, 9, 64, 128, 3, 1, True), (64, 7, 512, 512, 3, 1, True), (64, 28, 128, 128, 3, 1, True),
    (64, 14, 256, 1024, 1, 1, True), (64, 56, 128, 128, 3, 2, True),
    # N = 64 on the 256 x 128 tile (half the columns past N: the general epilogue), ragged
    (2, 56, 64, 64, 3, 1, True), (1, 9, 64, 64, 3, 1, True)])
def test_x3p_conv_stats(N, H, Cin, Cout, k, stride, pro):
    """Both operands pre-split (CAPMI_GEMM_X3P): the conv of relu(x*s+b) (split pass) vs fp64, and
    the BN statistics; ragged M (tiles of 256 rows), stream-K and data-parallel grids."""
    K = _K()
    pad = k // 2
    Ho = (H + 2 * pad - k) // stride + 1
    x = rnd(N, H, H, Cin, seed=11)
    w = rnd(Cout, k, k, Cin, seed=12) * (2.0 / (k * k * Cin)) ** 0.5
    s, b = rnd(Cin, seed=13) + 1.0, rnd(Cin, seed=14)
    xin = torch.relu(torch.addcmul(b, x, s)) if pro else x
    rows, Kd = N * Ho * Ho, k * k * Cin
    ws = K.gemm_workspace(DEV)
    xp = torch.empty(3 * x.numel(), device=DEV, dtype=torch.bfloat16)
    K.bn_relu_split3(x.to(DEV), s.to(DEV) if pro else None, b.to(DEV) if pro else None, N * H * H, Cin, xp)
    stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=DEV)
    out = torch.full((rows, Cout), float("nan"), device=DEV)
    w3 = split3(K.conv_weight_order_x3p(w.reshape(Cout, Kd), k, k, Cin).contiguous().to(DEV))
    if k == 1 and stride == 1:
        prob, mode = K.problem(rows, Cout, Kd, xp, Cin, w3, Kd, out, Cout, stats=stats), 0
    else:
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
        prob, mode = K.problem(rows, Cout, Kd, xp, 0, w3, Kd, out, Cout, conv=geo, stats=stats), 2
    K.gemm_x3p(prob, mode, ws)
    torch.cuda.synchronize()
    K.sk_check([ws])
    xi = xin.double().permute(0, 3, 1, 2)
    wt = w.double().permute(0, 3, 1, 2)
    ref = F.conv2d(xi, wt, stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    ref_abs = F.conv2d(xi.abs(), wt.abs(), stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    r3, _ = _errs(out, ref, ref_abs)
    assert r3 <= 1.0, r3
    o = out.double().cpu()
    st = stats.double().cpu()[: 2 * ((rows + 63) // 64) * Cout].view(-1, Cout, 2)
    torch.testing.assert_close(st[..., 0].sum(0), o.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(st[..., 1].sum(0), (o * o).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,H,Cin,Cout,k,stride,pro", [
    (4, 14, 256, 256, 3, 1, True), (4, 28, 128, 128, 3, 2, True), (2, 56, 64, 256, 1, 1, True),
    (3, 14, 256, 1024, 1, 1, True), (2, 7, 512, 2048, 1, 1, False), (64, 14, 256, 256, 3, 1, True),
    (1, 9, 64, 128, 3, 1, True), (64, 14, 1024, 256, 1, 1, False), (64, 28, 128, 128, 3, 1, True),
    (64, 14, 256, 1024, 1, 1, True), (64, 56, 128, 128, 3, 2, True), (64, 28, 512, 256, 1, 2, False)])
def test_x3d_conv_stats(N, H, Cin, Cout, k, stride, pro):
    """A fp32 split in-kernel with the BN prologue, B pre-split in the x3p order (CAPMI_GEMM_X3D):
    the conv of relu(x*s+b) vs fp64 under the x3 rule, and the BN statistics; dense 1x1 (no prologue,
    stride 1) through CAPMI_A_KMAJOR."""
    K = _K()
    pad = k // 2
    Ho = (H + 2 * pad - k) // stride + 1
    x = rnd(N, H, H, Cin, seed=21)
    w = rnd(Cout, k, k, Cin, seed=22) * (2.0 / (k * k * Cin)) ** 0.5
    s, b = rnd(Cin, seed=23) + 1.0, rnd(Cin, seed=24)
    xin = torch.relu(torch.addcmul(b, x, s)) if pro else x
    rows, Kd = N * Ho * Ho, k * k * Cin
    ws = K.gemm_workspace(DEV)
    xd = x.to(DEV).contiguous()
    stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=DEV)
    out = torch.full((rows, Cout), float("nan"), device=DEV)
    w3 = split3(K.conv_weight_order_x3p(w.reshape(Cout, Kd), k, k, Cin).contiguous().to(DEV))
    if k == 1 and stride == 1 and not pro:
        prob, mode = K.problem(rows, Cout, Kd, xd, Cin, w3, Kd, out, Cout, stats=stats), 0
    else:
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
        prob = K.problem(rows, Cout, Kd, xd, 0, w3, Kd, out, Cout, conv=geo, stats=stats,
                         in_scale=s.to(DEV) if pro else None, in_shift=b.to(DEV) if pro else None)
        mode = 2
    K.gemm_x3d(prob, mode, ws)
    torch.cuda.synchronize()
    K.sk_check([ws])
    xi = xin.double().permute(0, 3, 1, 2)
    wt = w.double().permute(0, 3, 1, 2)
    ref = F.conv2d(xi, wt, stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    ref_abs = F.conv2d(xi.abs(), wt.abs(), stride=stride, padding=pad).permute(0, 2, 3, 1).reshape(rows, Cout)
    r3, _ = _errs(out, ref, ref_abs)
    assert r3 <= 1.0, r3
    o = out.double().cpu()
    st = stats.double().cpu()[: 2 * ((rows + 63) // 64) * Cout].view(-1, Cout, 2)
    torch.testing.assert_close(st[..., 0].sum(0), o.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(st[..., 1].sum(0), (o * o).sum(0), rtol=1e-5, atol=1e-3)


def test_encoder_x3_oversize_batch_routes_to_fp32():
    """A per-GPU batch whose conv input passes 2 GiB (layer1's 56x56x256 fp32 map at B = 672: 2.16e9 B)
    exceeds the x3 kernels' 32-bit buffer offsets: those convs run the fp32 MFMA kernel instead of the
    planner raising CAPMI_ERANGE (capmi.resnet.EncoderRunner._conv); the rest stay x3. The features
    must match the all-fp32 encoder's to the two paths' fp32-level accuracy."""
    import gen
    from helpers import rel_err, t
    from capmi.resnet import EncoderRunner, ResNet101
    B = 672
    net = ResNet101()
    sd = net.state_dict()
    for k_, v in gen.resnet101_params(79).items():
        sd[k_] = t(v).clone()
    net.load_state_dict(sd)
    net = net.to(DEV).train()
    x = t(gen.images(79, 8), DEV).repeat(B // 8, 1, 1, 1).contiguous()  # 0.4 GB of 224^2 images
    r3, r1 = EncoderRunner(), EncoderRunner()
    r3.x3 = True
    with torch.no_grad():
        y3 = r3.forward(net, x, out_hw=None)
        y1 = r1.forward(net, x, out_hw=None)
    torch.cuda.synchronize()
    assert torch.isfinite(y3).all()
    assert rel_err(y3, y1) < 5e-3, rel_err(y3, y1)


@pytest.mark.parametrize("N,H,Cout,pro,lda", [
    (2, 56, 256, True, 0), (2, 56, 64, False, 0), (1, 11, 256, True, 0), (3, 7, 128, False, 80),
    (1, 9, 64, True, 0), (64, 56, 256, True, 0), (64, 56, 64, False, 64)])
def test_x3s_short_k(N, H, Cout, pro, lda):
    """The short-k streaming kernel (CAPMI_GEMM_X3S, layer1's K = 64 convs): the 1x1 conv of
    relu(x*s+b) (or dense rows of stride lda) vs fp64 under the x3 rule, the BN statistics of the
    stored output, and nothing written past row M (NaN sentinel rows after C)."""
    K = _K()
    Cin = 64
    rows = N * H * H
    x = rnd(rows, max(lda, Cin), seed=31)
    w = rnd(Cout, Cin, seed=32) * (2.0 / Cin) ** 0.5
    s, b = rnd(Cin, seed=33) + 1.0, rnd(Cin, seed=34)
    xin = torch.relu(torch.addcmul(b, x[:, :Cin], s)) if pro else x[:, :Cin]
    stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=DEV)
    buf = torch.full((rows + 64, Cout), float("nan"), device=DEV)
    out = buf[:rows]
    xd = x.to(DEV).contiguous()
    w3, sd, bd = split3(w.to(DEV)), s.to(DEV), b.to(DEV)  # held until the launch has run (raw pointers)
    if lda:
        prob, mode = K.problem(rows, Cout, Cin, xd, lda, w3, Cin, out, Cout, stats=stats), 0
    else:
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=1, KW=1, stride=1, pad=0, Ho=H, Wo=H)
        prob = K.problem(rows, Cout, Cin, xd, 0, w3, Cin, out, Cout, conv=geo, stats=stats,
                         in_scale=sd if pro else None, in_shift=bd if pro else None)
        mode = 2
    assert K.gemm_x3s_ok(prob, mode)
    K.gemm_x3s(prob, mode)
    torch.cuda.synchronize()
    ref = xin.double() @ w.double().T
    ref_abs = xin.double().abs() @ w.double().abs().T
    r3, _ = _errs(out, ref, ref_abs)
    assert r3 <= 1.0, r3
    assert bool(torch.isnan(buf[rows:]).all()), "x3s wrote past row M"
    o = out.double().cpu()
    st = stats.double().cpu().view(-1, Cout, 2)
    torch.testing.assert_close(st[..., 0].sum(0), o.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(st[..., 1].sum(0), (o * o).sum(0), rtol=1e-5, atol=1e-3)
    # each 64-row slice's statistics are that slice's sums (what bn_finalize reads)
    sl = torch.nn.functional.pad(o, (0, 0, 0, (-rows) % 64)).view(-1, 64, Cout)
    torch.testing.assert_close(st[..., 0], sl.sum(1), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N,H,Cin,Cout", [(64, 14, 256, 1024), (3, 7, 512, 2048), (1, 9, 64, 128)])
def test_x3d_dense_prologue_equals_conv_form(N, H, Cin, Cout):
    """x3d on a 1x1 conv's input as dense rows with the BN prologue (k = channel; round 3) == the same
    conv through the implicit-im2col form, bit for bit (output and BN statistics)."""
    K = _K()
    rows = N * H * H
    x = rnd(rows, Cin, seed=51).to(DEV)
    s, b = (rnd(Cin, seed=52) + 1.0).to(DEV), rnd(Cin, seed=53).to(DEV)
    w3 = split3((rnd(Cout, Cin, seed=54) * (2.0 / Cin) ** 0.5).to(DEV))
    ws = K.gemm_workspace(DEV)
    geo = dict(N=N, H=H, W=H, Cin=Cin, KH=1, KW=1, stride=1, pad=0, Ho=H, Wo=H)
    outs = []
    for dense in (True, False):
        out = torch.empty(rows, Cout, device=DEV)
        st = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=DEV)
        if dense:
            prob = K.problem(rows, Cout, Cin, x, Cin, w3, Cin, out, Cout, stats=st, in_scale=s, in_shift=b)
        else:
            prob = K.problem(rows, Cout, Cin, x, 0, w3, Cin, out, Cout, stats=st, conv=geo, in_scale=s, in_shift=b)
        K.gemm_x3d(prob, 0 if dense else 2, ws)
        outs.append((out, st))
    torch.cuda.synchronize()
    K.sk_check([ws])
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_x3d_prologue_scale_shift_at_allocation_end():
    """VERDICT r2 weak 12 (the over-read class of the round-2 x3d fault): the BN scale / shift are the LAST
    Cin floats of their buffers, followed only by NaN sentinels in the same allocation; the x3d prologue reads
    them through descriptors sized to Cin, so the result equals the one with padded copies bit for bit and no
    NaN reaches the output (a stride-2 3x3 and a 1x1 conv input, batch 2)."""
    K = _K()
    ws = K.gemm_workspace(DEV)
    for (N, H, Cin, Cout, k, stride) in [(2, 28, 128, 256, 3, 2), (2, 14, 256, 1024, 1, 1)]:
        pad = k // 2
        Ho = (H + 2 * pad - k) // stride + 1
        rows, Kd = N * Ho * Ho, k * k * Cin
        x = rnd(N * H * H, Cin, seed=61).to(DEV)
        s, b = (rnd(Cin, seed=62) + 1.0).to(DEV), rnd(Cin, seed=63).to(DEV)
        tail = torch.full((2, Cin + 64), float("nan"), device=DEV)  # [scale | NaN x 64], [shift | NaN x 64]
        tail[0, :Cin], tail[1, :Cin] = s, b
        w3 = split3(K.conv_weight_order_x3p((rnd(Cout, Kd, seed=64) * (2.0 / Kd) ** 0.5).to(DEV), k, k, Cin)
                    .contiguous())
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Ho)
        outs = []
        for sc, sh in ((s.clone(), b.clone()), (tail[0, :Cin], tail[1, :Cin])):
            out = torch.empty(rows, Cout, device=DEV)
            if k == 1 and stride == 1:
                prob, mode = K.problem(rows, Cout, Kd, x, Cin, w3, Kd, out, Cout, in_scale=sc, in_shift=sh), 0
            else:
                prob, mode = K.problem(rows, Cout, Kd, x, 0, w3, Kd, out, Cout, conv=geo, in_scale=sc, in_shift=sh), 2
            K.gemm_x3d(prob, mode, ws)
            outs.append(out)
        torch.cuda.synchronize()
        K.sk_check([ws])
        assert bool(torch.isfinite(outs[1]).all())
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,H,Cin,pro", [(2, 56, 64, True), (64, 56, 64, True), (3, 14, 64, True), (1, 9, 64, False),
                                         (2, 20, 96, True), (5, 7, 32, True), (1, 64, 64, False)])
def test_x3c_direct_conv(N, H, Cin, pro):
    """CAPMI_GEMM_X3C (round 4): the direct 3x3 / stride-1 conv of layer1 (Cout 64) within the x3 bound of the
    fp64 conv (the rule of test_x3_conv_prologue_stats), equal to gemm_x3p on the split input planes up to the
    order of its k-split partial sums (rel L2 <= 1e-6), its per-64-row BN statistics those of its own output,
    and no store past M (NaN sentinels); tiles straddling image boundaries (H = 14, 9, 7), a ragged last tile,
    Cin = 32 / 96, W = 64 (the kernel's bound), with and without the BN-apply + ReLU prologue."""
    K = _K()
    Cout, k = 64, 3
    rows, Kd = N * H * H, 9 * Cin
    x = rnd(N, H, H, Cin, seed=71)
    w = rnd(Cout, k, k, Cin, seed=72) * (2.0 / Kd) ** 0.5
    s, b = rnd(Cin, seed=73) + 1.0, rnd(Cin, seed=74)
    xd, sd, bd = x.to(DEV), s.to(DEV), b.to(DEV)
    w3 = split3(K.conv_weight_order_x3p(w.reshape(Cout, Kd).to(DEV), k, k, Cin).contiguous())
    geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=1, pad=1, Ho=H, Wo=H)
    ws = K.gemm_workspace(DEV)
    T = (rows + 63) // 64
    out_c, st_c = torch.full((rows + 5, Cout), float("nan"), device=DEV), torch.zeros(2 * T * Cout, device=DEV)
    pc = K.problem(rows, Cout, Kd, xd, 0, w3, Kd, out_c, Cout, conv=geo, stats=st_c,
                   in_scale=sd if pro else None, in_shift=bd if pro else None)
    assert K.gemm_x3c_ok(pc)
    K.gemm_x3c(pc)
    # gemm_x3p on the same split input planes
    xp = torch.empty(3 * rows * Cin, device=DEV, dtype=torch.bfloat16)
    K.bn_relu_split3(xd, sd if pro else None, bd if pro else None, rows, Cin, xp)
    out_p, st_p = torch.empty(rows, Cout, device=DEV), torch.zeros(2 * T * Cout, device=DEV)
    pp = K.problem(rows, Cout, Kd, xp, 0, w3, Kd, out_p, Cout, conv=geo, stats=st_p)
    K.gemm_x3p(pp, 2, ws)
    torch.cuda.synchronize()
    K.sk_check([ws])
    assert bool(torch.isnan(out_c[rows:]).all())
    oc = out_c[:rows].double().cpu()
    assert float((oc - out_p.double().cpu()).norm() / out_p.double().cpu().norm()) <= 1e-6
    sl = torch.nn.functional.pad(oc, (0, 0, 0, T * 64 - rows)).view(T, 64, Cout)
    st = st_c.double().cpu().view(T, Cout, 2)
    torch.testing.assert_close(st[..., 0], sl.sum(1), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(st[..., 1], (sl * sl).sum(1), rtol=1e-5, atol=1e-4)
    xin = torch.relu(x * s + b) if pro else x
    xi, wt = xin.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2)
    ref = F.conv2d(xi, wt, padding=1).permute(0, 2, 3, 1).reshape(rows, Cout)
    ref_abs = F.conv2d(xi.abs(), wt.abs(), padding=1).permute(0, 2, 3, 1).reshape(rows, Cout)
    r3, _ = _errs(out_c[:rows], ref, ref_abs)
    assert r3 <= 1.0, r3


@pytest.mark.parametrize("M,N,Kd", [(12544, 1024, 256), (3137, 256, 512), (777, 128, 64 * 9)])
def test_beta_epilogue_batched_loads(M, N, Kd):
    """C = A.B + beta C (the store-only epilogue with beta, round 4: C loaded ahead of the stores) on x3d (dense
    rows, data-parallel for beta problems) and gemm_x3: bit-identical to the product (beta onto zeros) plus C0 in
    fp32 (fmaf(1, c, v) rounds v + c once), rows past M untouched (NaN sentinels)."""
    K = _K()
    A, W = rnd(M, Kd, seed=91), rnd(N, Kd, seed=92)
    C0 = rnd(M, N, seed=93)
    Ad, w3 = A.to(DEV), split3(W.to(DEV))
    ws = K.gemm_workspace(DEV)
    for name in ("x3d", "x3"):
        run = (lambda p: K.gemm_x3d(p, 0, ws)) if name == "x3d" else (lambda p: K.gemm_x3(p, 0, ws))
        c_beta = torch.full((M + 3, N), float("nan"), device=DEV)
        c_beta[:M] = C0.to(DEV)
        run(K.problem(M, N, Kd, Ad, Kd, w3, Kd, c_beta, N, beta=1.0))
        # the reference with the same schedule (x3d takes beta problems data-parallel, plain ones stream-K):
        # beta = 1 onto zeros, fmaf(1, 0, v) = v
        c_plain = torch.zeros(M, N, device=DEV)
        run(K.problem(M, N, Kd, Ad, Kd, w3, Kd, c_plain, N, beta=1.0))
        torch.cuda.synchronize()
        K.sk_check([ws])
        assert torch.equal(c_beta[:M].cpu(), c_plain.cpu() + C0), name
        assert bool(torch.isnan(c_beta[M:]).all()), name
