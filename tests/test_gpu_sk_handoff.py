"""GPU: the stream-K hand-off of the one-workgroup-per-CU x3 kernels (x3p, x3d, gemm_x3) under uneven load.

Round 5 dropped the agent-scope release / acquire fences from these kernels' hand-off and relies on the form
MI355X_MICROARCH.md lists as measured-valid (table row 1 of "Valid forms besides Guideline 16", restated with
its four conditions in DESIGN.md §4.14 and csrc/gemm_args.h): sc1 partial stores drained by every wave, a
barrier, ONE lane's sc1 flag store; the owner polls the flag with sc1 loads and its waves read the partial
with sc1 loads behind a barrier. The guide asks such a hand-off to be tested under UNEVEN load with the
consumer L1-warm, checking every word. Every launch below runs while another stream keeps part of the chip
busy and re-uses the same parked-partial slots. ADVICE r5: consecutive launches alternate between two input
sets whose results differ everywhere, so a stale partial left by the previous launch (of the OTHER input)
would show; each result must equal the one its own input gave in a quiet launch bit for bit (the partials
are added in a fixed order), that quiet result must match an fp64 reference, and no flag may stay raised."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
RUNS = 24


def _K():
    from capmi import kernels as K
    return K


def _case(kind, seed):
    """(run, outputs, workspace, fp64 reference) of one stream-K launch at the encoder's batch-64 shapes;
    ``seed`` picks the input (activations, BN scale / shift); the weight is shared."""
    K = _K()
    gw = torch.Generator(device=DEV).manual_seed(7)
    g = torch.Generator(device=DEV).manual_seed(100 + seed)
    if kind == "x3p":  # layer3 3x3 conv on pre-split planes: 98 tiles x 72 k-tiles over every CU
        N, H, ci, co, k = 64, 14, 256, 256, 3
    elif kind == "x3d":  # layer3 c3 as dense rows with the BN prologue: 392 tiles x 8 k-tiles
        N, H, ci, co, k = 64, 14, 256, 1024, 1
    else:  # gemm_x3 on a layer4-sized 1x1 (50 tiles of 128 x 128: stream-K even with the family data-parallel)
        N, H, ci, co, k = 64, 7, 2048, 256, 1
    M, Kd = N * H * H, ci * k * k
    w = torch.rand(co, Kd, device=DEV, generator=gw) - 0.5
    x = torch.rand(N, H, H, ci, device=DEV, generator=g) - 0.5
    sc = torch.rand(ci, device=DEV, generator=g) + 0.5
    sh = torch.rand(ci, device=DEV, generator=g) - 0.5
    y = torch.empty(M, co, device=DEV)
    stats = torch.zeros(K.stat_tiles(M, 1) * co * 2 + 64, device=DEV)
    w3 = torch.empty(3 * w.numel(), device=DEV, dtype=torch.bfloat16)
    x64 = x.double()
    if kind != "x3":
        x64 = torch.relu(x64 * sc.double() + sh.double())
    if kind == "x3p":
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, ci).contiguous(), w3)
        xp = torch.empty(3 * x.numel(), device=DEV, dtype=torch.bfloat16)
        K.bn_relu_split3(x, sc, sh, x.numel() // ci, ci, xp)
        geo = dict(N=N, H=H, W=H, Cin=ci, KH=k, KW=k, stride=1, pad=k // 2, Ho=H, Wo=H)
        prob = K.problem(M, co, Kd, xp, 0, w3, Kd, y, co, conv=geo, stats=stats)
        assert K.gemm_x3p_kernel_name(prob, 2).startswith("gemm_x3p_kernel<2, true")
        run = lambda ws: K.gemm_x3p(prob, 2, ws)  # noqa: E731
        keep = (xp,)
        # fp64 im2col + GEMM on the device (unfold's k order is (ci, kh, kw))
        cols = torch.nn.functional.unfold(x64.permute(0, 3, 1, 2), k, padding=k // 2)  # (N, ci k k, H W)
        w4 = w.double().view(co, k, k, ci).permute(0, 3, 1, 2).reshape(co, Kd)
        ref = (w4 @ cols).permute(0, 2, 1).reshape(M, co)
    elif kind == "x3d":
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, ci).contiguous(), w3)
        prob = K.problem(M, co, Kd, x, ci, w3, Kd, y, co, stats=stats, in_scale=sc, in_shift=sh)
        assert K.gemm_x3d_kernel_name(prob, 0).startswith("gemm_x3p_kernel<0, true")
        run = lambda ws: K.gemm_x3d(prob, 0, ws)  # noqa: E731
        keep = ()
        ref = x64.reshape(M, ci) @ w.double().t()
    else:
        K.split3_bf16(w, w3)
        prob = K.problem(M, co, Kd, x, ci, w3, Kd, y, co, stats=stats)
        assert K.gemm_x3_kernel_name(prob, 0).endswith("true>")
        run = lambda ws: K.gemm_x3(prob, 0, ws)  # noqa: E731
        keep = ()
        ref = x64.reshape(M, ci) @ w.double().t()
    nst = K.stat_tiles(M, 1) * co * 2
    return (lambda ws: (run(ws), keep, x, w3, sc, sh)[0]), (y, stats[:nst]), ref


@pytest.mark.parametrize("kind", ["x3p", "x3d", "x3"])
def test_sk_handoff_uneven_load_bit_stable(kind):
    K = _K()
    ws = K.gemm_workspace(DEV)  # one set of parked-partial slots and flags for both inputs
    cases = [_case(kind, s) for s in (0, 1)]
    quiet = []
    for run, (y, stats), ref in cases:
        run(ws)
        torch.cuda.synchronize()
        K.sk_check([ws])
        err = float((y.double() - ref).norm() / ref.norm())
        assert err < 1e-5, (kind, err)  # the x3 arithmetic is fp32-accurate; a stale partial is O(1)
        quiet.append((y.clone(), stats.clone()))
    assert not torch.equal(quiet[0][0], quiet[1][0])
    # the load: a long stream of matmuls on a second stream whose blocks hold some CUs while the GEMM runs, so
    # stream-K workers start and reach their hand-offs at uneven times
    side = torch.cuda.Stream()
    a = torch.rand(2048, 2048, device=DEV)
    for r in range(RUNS):
        c = r % 2
        run, (y, stats), _ = cases[c]
        y.fill_(float("nan"))
        stats.fill_(float("nan"))
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(1 + r % 4):
                a = (a @ a).clamp_(-1, 1)
        run(ws)
        torch.cuda.synchronize()
        K.sk_check([ws])
        y0, s0 = quiet[c]
        assert torch.equal(y, y0), (kind, r, int((y != y0).sum()))
        assert torch.equal(stats, s0), (kind, r)
