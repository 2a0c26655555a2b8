"""GPU: train-mode BatchNorm finalize (models/encoder.py:97-107 -- torchvision BN in train mode, the reference
calls encoder.train(), models/attention.py:374) in its round-4 form: capmi_bn_finalize sums the per-slice
statistics in one canonical fp64 order (csrc/bn_final.h) and rounds every operation on its own, so its outputs
are reproduced BIT FOR BIT by the numpy restatement below."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    from capmi import kernels as K
    return K


def bn_final_ref(stats, count, gamma, beta, rm, rv, momentum, eps):
    """numpy restatement of csrc/bn_final.h (bnf_group + bnf_apply): q_l = sum over slices t = l (mod 64) in
    ascending t, r_w = q_8w + ... + q_8w+7, sum = r_0 + ... + r_7 (fp64, each sequential), then the finalize
    arithmetic op by op."""
    st = stats.astype(np.float64)  # (T, C, 2)
    T, C, _ = st.shape
    q = []
    for l_ in range(64):
        acc = np.zeros((C, 2))
        for t in range(l_, T, 64):
            acc = acc + st[t]
        q.append(acc)
    tot = np.zeros((C, 2))
    for w in range(8):
        r = np.zeros((C, 2))
        for s8 in range(8):
            r = r + q[8 * w + s8]
        tot = tot + r
    n = float(count)
    mean = tot[:, 0] / n
    var = tot[:, 1] / n - mean * mean
    var = np.where(var < 0, 0.0, var)
    inv = 1.0 / np.sqrt(var + np.float64(np.float32(eps)))
    sc = (gamma.astype(np.float64) * inv).astype(np.float32)
    sh = (beta.astype(np.float64) - mean * sc.astype(np.float64)).astype(np.float32)
    unb = var * n / (n - 1.0) if count > 1 else var
    m = np.float32(momentum)
    one_m = np.float32(1.0) - m
    rm2 = one_m * rm.astype(np.float32) + m * mean.astype(np.float32)
    rv2 = one_m * rv.astype(np.float32) + m * unb.astype(np.float32)
    return sc, sh, mean.astype(np.float32), var.astype(np.float32), rm2, rv2


@pytest.mark.parametrize("C,T,count", [(64, 3136, 200704), (2048, 49, 3136), (256, 196, 12544), (1024, 7, 420),
                                       (512, 256, 16384), (128, 257, 16400), (20, 3, 130), (64, 12544, 802816)])
def test_bn_finalize_canonical_order(C, T, count):
    """capmi_bn_finalize == the numpy restatement, bit for bit (scale, shift, batch mean / var, running stats),
    and within fp64 rounding of torch's own batch statistics."""
    K = _K()
    g = torch.Generator().manual_seed(C + T)
    x = torch.randn(T * 64, C, generator=g, dtype=torch.float64) * 3 + 1
    stats = torch.stack([x.view(T, 64, C).sum(1), (x * x).view(T, 64, C).sum(1)], -1).float()
    gamma, beta = (torch.rand(C, generator=g) + 0.5).float(), torch.randn(C, generator=g).float()
    rm, rv = torch.randn(C, generator=g).float(), (torch.rand(C, generator=g) + 0.5).float()
    sd = [t.to(DEV) for t in (stats, gamma, beta, rm, rv)]
    scale, shift = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    mean, var = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    work = torch.zeros(K.bn_work_doubles(C), device=DEV, dtype=torch.float64)
    K.bn_finalize(sd[0], T, C, count, sd[1], sd[2], sd[3], sd[4], 0.1, 1e-5, scale, shift, work,
                  save_mean=mean, save_var=var)
    torch.cuda.synchronize()
    ref = bn_final_ref(stats.numpy(), count, gamma.numpy(), beta.numpy(), rm.numpy(), rv.numpy(), 0.1, 1e-5)
    for name, got, want in zip(("scale", "shift", "mean", "var", "running_mean", "running_var"),
                               (scale, shift, mean, var, sd[3], sd[4]), ref):
        assert np.array_equal(got.cpu().numpy(), want), name
    if count == T * 64:  # the statistics of x itself: torch's fp64 batch mean / var
        torch.testing.assert_close(mean.double().cpu(), x.mean(0), rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(var.double().cpu(), x.var(0, unbiased=False), rtol=1e-5, atol=1e-6)
