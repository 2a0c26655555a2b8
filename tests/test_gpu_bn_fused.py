"""GPU: capmi_bn_finalize_apply (the train-mode BN finalize fused into its consumer pass; opt-in,
CAPMI_BN_FUSE=1) against
the two-launch path it replaces (capmi_bn_finalize + bn_relu_split3 / bn_add_relu / bn_relu_bf16 /
bn_add_relu_bf16) on the same slice statistics.

The finalize sums the same fp64 partials in a different fixed order, so scale / shift / running
statistics agree to fp32 rounding (rel. 1e-6), the fp32 outputs to that times |y| (rel. 1e-5), and
the bf16 outputs to one bf16 ulp. The running statistics must be updated exactly once (one
momentum step), whatever the number of row chunks."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    from capmi import kernels as K
    return K


def _setup(rows, C, seed):
    g = torch.Generator().manual_seed(seed)
    y = (torch.randn(rows, C, generator=g) * 2 + 0.5).float()
    tiles = (rows + 63) // 64
    yp = torch.zeros(tiles * 64, C)
    yp[:rows] = y
    yd = yp.view(tiles, 64, C).double()
    stats = torch.stack([yd.sum(1), (yd * yd).sum(1)], -1).float()  # [tiles][C][2], as the GEMM epilogue
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    rm, rv = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    res = torch.randn(rows, C, generator=g)
    return [t.to(DEV).contiguous() for t in (y, stats, gamma, beta, rm, rv, res)], tiles


def _ref_finalize(K, stats, tiles, C, rows, gamma, beta, rm, rv):
    s, b = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    work = torch.zeros(K.bn_work_doubles(C), device=DEV, dtype=torch.float64)
    K.bn_finalize(stats, tiles, C, rows, gamma, beta, rm2, rv2, 0.1, 1e-5, s, b, work)
    return s, b, rm2, rv2


def _close(a, b, rtol, what, atol=0.0):
    a, b = a.double().cpu(), b.double().cpu()
    err = (a - b).abs()
    tol = rtol * b.abs() + atol
    assert bool((err <= tol).all()), f"{what}: max err {float(err.max()):.3g}"


@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("rows,C", [(12544, 256), (3136, 1024), (1000, 64)])
def test_bn_finalize_apply_matches_two_launch_path(op, rows, C):
    K = _K()
    (y, stats, gamma, beta, rm, rv, res), tiles = _setup(rows, C, 3 + op)
    s_ref, b_ref, rm_ref, rv_ref = _ref_finalize(K, stats, tiles, C, rows, gamma, beta, rm, rv)
    s, b = torch.full((C,), float("nan"), device=DEV), torch.full((C,), float("nan"), device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    bf = torch.bfloat16
    if op == 0:
        out = torch.empty(3 * rows * C, device=DEV, dtype=bf)
        K.bn_finalize_apply(0, stats, tiles, C, rows, gamma, beta, rm2, rv2, 0.1, 1e-5, s, b, y, out, rows)
        ref = torch.empty(3 * rows * C, device=DEV, dtype=bf)
        K.bn_relu_split3(y, s_ref, b_ref, rows, C, ref)
        got = out.view(3, -1).float().sum(0)  # the three planes sum exactly to the fp32 value
        want = ref.view(3, -1).float().sum(0)
        _close(got, want, 1e-5, "split3 value", atol=1e-6)
    elif op == 1:
        out = torch.empty(rows, C, device=DEV)
        K.bn_finalize_apply(1, stats, tiles, C, rows, gamma, beta, rm2, rv2, 0.1, 1e-5, s, b, y, out, rows, res=res)
        ref = torch.empty(rows, C, device=DEV)
        K.bn_add_relu(y, s_ref, b_ref, res, ref, rows, C)
        _close(out, ref, 1e-5, "add_relu", atol=1e-5)
    else:
        yb, rb = y.to(bf), res.to(bf)
        out = torch.empty(rows, C, device=DEV, dtype=bf)
        ref = torch.empty(rows, C, device=DEV, dtype=bf)
        if op == 2:
            yin = yb.clone()
            K.bn_finalize_apply(2, stats, tiles, C, rows, gamma, beta, rm2, rv2, 0.1, 1e-5, s, b, yin, yin, rows)
            out = yin  # in place
            K.bn_relu_bf16(yb, s_ref, b_ref, rows, C, ref)
        else:
            K.bn_finalize_apply(3, stats, tiles, C, rows, gamma, beta, rm2, rv2, 0.1, 1e-5, s, b, yb, out, rows,
                                res=rb)
            K.bn_add_relu_bf16(yb, s_ref, b_ref, rb, ref, rows, C)
        _close(out.float(), ref.float(), 2.0 ** -7, "bf16 apply", atol=1e-2)
        assert float((out.float() == ref.float()).float().mean()) > 0.99
    _close(s, s_ref, 1e-6, "scale")
    _close(b, b_ref, 1e-6, "shift", atol=1e-7)
    _close(rm2, rm_ref, 1e-6, "running_mean", atol=1e-7)  # one momentum step, not one per chunk
    _close(rv2, rv_ref, 1e-6, "running_var")


def test_bn_finalize_apply_rejects_large_tiles():
    from capmi._lib import CapmiError
    K = _K()
    (y, stats, gamma, beta, rm, rv, res), tiles = _setup(64 * 300, 32, 9)
    s, b = torch.empty(32, device=DEV), torch.empty(32, device=DEV)
    out = torch.empty(64 * 300, 32, device=DEV)
    with pytest.raises(CapmiError):
        K.bn_finalize_apply(1, stats, tiles, 32, 64 * 300, gamma, beta, rm, rv, 0.1, 1e-5, s, b, y, out, 64 * 300,
                            res=res)
