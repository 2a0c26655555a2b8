"""GPU: the baseline decoder (reference models/baseline.py:24-111) on the capmi kernels
(capmi/baseline_fn.py).

* forward against the reference's own golden scores (tests/golden/baseline_forward.npz, made by
  the real reference module): rtol 1e-4 / atol 1e-5 (fp32, different summation order);
* forward + backward against the oracle's math (oracle.decoder_ref.baseline_forward, pinned to
  that golden by test_oracle_golden.py; restated below without its fp32 casts) evaluated in fp64
  by autograd, with the reference's loss (CE, ignore_index = PAD, against the captions incl. <start>), at the
  golden size and at the production size (L = 25, M = H = 512, V = 8100): scores rel. L2 <= 1e-5,
  every parameter gradient and d(img_features) rel. L2 <= 1e-4 (fp32 BPTT vs fp64).
"""
import numpy as np
import pytest
import torch

import gen
from helpers import rel_err, t
from oracle import decoder_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ["embedding.weight", "lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0",
         "linear.weight", "linear.bias"]


def _decoder(B, L, M, H, V, s, device):
    from models.baseline import BaselineDecoder, BaselineDecoderParams
    prm = BaselineDecoderParams()
    prm.embed_size, prm.hidden_size, prm.vocab_size = M, H, V
    dec = BaselineDecoder(prm)
    shapes = {"embedding.weight": (V, M), "lstm.weight_ih_l0": (4 * H, M), "lstm.weight_hh_l0": (4 * H, H),
              "lstm.bias_ih_l0": (4 * H,), "lstm.bias_hh_l0": (4 * H,), "linear.weight": (V, H),
              "linear.bias": (V,)}
    p = {k: t(gen.uniform(s, k, v, -0.2, 0.2)) for k, v in shapes.items()}
    dec.load_state_dict(p)
    feats = t(gen.uniform(s, "feats", (B, M), -1, 1))
    return dec.to(device), p, feats


def _forward64(p, feats, caps):
    """oracle.decoder_ref.baseline_forward in fp64 (same ops: embedding of captions[:, :-1] after
    the image feature, torch LSTM cell i,f,g,o, Linear)."""
    x = torch.cat((feats.unsqueeze(1), torch.nn.functional.embedding(caps[:, :-1], p["embedding.weight"])), 1)
    B, L, _ = x.shape
    H = p["lstm.weight_hh_l0"].shape[1]
    h = torch.zeros(B, H, dtype=torch.float64)
    c = torch.zeros(B, H, dtype=torch.float64)
    outs = []
    for step in range(L):
        g = (x[:, step] @ p["lstm.weight_ih_l0"].T + p["lstm.bias_ih_l0"] + h @ p["lstm.weight_hh_l0"].T
             + p["lstm.bias_hh_l0"])
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs.append(h)
    return torch.nn.functional.linear(torch.stack(outs, 1), p["linear.weight"], p["linear.bias"])


def test_baseline_forward_vs_reference_golden(golden):
    fx = golden("baseline_forward")
    m = fx["meta"]
    dec, _, feats = _decoder(m["B"], m["L"], m["M"], m["H"], m["V"], m["seed"], DEV)
    with torch.no_grad():
        scores = dec(feats.to(DEV), t(fx["captions"], DEV))
    torch.cuda.synchronize()
    np.testing.assert_allclose(scores.cpu().numpy(), fx["scores"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,L,M,H,V,pad", [(4, 9, 16, 24, 40, True), (4, 25, 512, 512, 8100, False)])
def test_baseline_train_step_vs_oracle_fp64(B, L, M, H, V, pad):
    dec, p, feats = _decoder(B, L, M, H, V, 5, DEV)
    g = torch.Generator().manual_seed(7)
    caps = torch.randint(1, V, (B, L), generator=g)
    if pad:  # ragged captions padded with PAD = 0 (ignored by the loss, still fed as inputs)
        caps[1, 6:] = 0
        caps[3, 4:] = 0
    # reference: the oracle in fp64 under autograd
    p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
    f64 = feats.double().requires_grad_(True)
    R_scores = _forward64(p64, f64, caps)
    loss64 = R.baseline_loss(R_scores, caps)
    loss64.backward()
    # capmi
    fd = feats.to(DEV).requires_grad_(True)
    scores = dec(fd, caps.to(DEV))
    loss = torch.nn.functional.cross_entropy(scores.reshape(-1, V), caps.to(DEV).reshape(-1), ignore_index=0)
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(scores, R_scores.detach()) < 1e-5, rel_err(scores, R_scores.detach())
    grads = dict(dec.named_parameters())
    for k in NAMES:
        e = rel_err(grads[k].grad, p64[k].grad)
        assert e < 1e-4, (k, e)
    assert rel_err(fd.grad, f64.grad) < 1e-4, rel_err(fd.grad, f64.grad)
