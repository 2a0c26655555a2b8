"""GPU: the fused recurrence kernels (csrc/decoder_step.hip, three launches per timestep each way)
against the generic per-op path (five launches per timestep, CAPMI_DEC_FUSED=0) and against fp64.

* capmi_dstep_gemm, every epilogue mode, against a torch fp64 reference of the same arithmetic
  (multi-segment K, gate-interleaved tiles, several row tiles, k-splits from 1 to 64 so the
  last-arriver reduction is exercised with and without parked partials);
* the whole decoder training step (loss, predictions, alphas, every gradient, d(encoder_out)) with
  the fused loop vs the generic loop: the same arithmetic in a different fp32 summation order, so
  rel. 2e-5 of max|.| per tensor; at the headline size (B = 64, ragged lengths), the BERT-feature
  width (M = 768), the GloVe width (M = 300), distinct rows (dup = 2) and B = 70 (two row tiles).
The oracle parity of the fused path itself is test_gpu_decoder.py / test_gpu_headline_parity.py
(the fused loop is the default)."""
import os

import numpy as np
import pytest
import torch

import gen
from helpers import make_decoder, t

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _sig(x):
    return 1.0 / (1.0 + torch.exp(-x))


@pytest.mark.parametrize("S", [1, 3, 8, 64])
def test_dstep_gemm_modes_vs_fp64(S):
    from capmi import kernels as K
    from capmi._lib import CAPMI_DSTEP_GATE_BWD, CAPMI_DSTEP_LSTM_BWD, CAPMI_DSTEP_LSTM_FWD, CAPMI_DSTEP_STORE2
    g = torch.Generator().manual_seed(S)
    Bm, D, E = 70, 64, 256

    def r(*s):
        return (torch.randn(*s, generator=g) * 0.5).to(DEV)

    part = torch.empty(1 << 22, device=DEV)
    cnt = torch.zeros(4096, device=DEV, dtype=torch.int32)
    # STORE2 over three K segments: columns [0, 96) + bias, [96, 160) sigmoid(. + bias)
    A1, A2, A3 = r(Bm, 64), r(Bm, 128), r(Bm, 32)
    W = r(160, 64 + 128 + 32)
    b0, b1 = r(96), r(64)
    o0, o1 = torch.empty(Bm, 96, device=DEV), torch.empty(Bm, 64, device=DEV)
    K.dstep_gemm([(A1, 64, W, 224, 64), (A2, 128, W[:, 64:], 224, 128), (A3, 32, W[:, 192:], 224, 32)],
                 Bm, 160, 32, S, dict(mode=CAPMI_DSTEP_STORE2, out0=o0, ld0=96, bias0=b0, nsplit=96, out1=o1,
                                      ld1=64, bias1=b1, act1=1), part, cnt)
    ref = torch.cat([A1, A2, A3], 1).double() @ W.double().T
    assert _rel(o0, ref[:, :96] + b0.double()) < 2e-6
    assert _rel(o1, _sig(ref[:, 96:] + b1.double())) < 2e-6
    # LSTM forward, gate-interleaved 64-column tiles
    x, h, c = r(Bm, E), r(Bm, D), r(Bm, D)
    Wx, Wh, xe = r(4 * D, E) * 0.1, r(4 * D, D) * 0.1, r(Bm, 4 * D)
    ho, co, act = torch.empty(Bm, D, device=DEV), torch.empty(Bm, D, device=DEV), torch.empty(Bm, 4 * D, device=DEV)
    K.dstep_gemm([(x, E, Wx, E, E), (h, D, Wh, D, D)], Bm, 4 * D, 64, S,
                 dict(mode=CAPMI_DSTEP_LSTM_FWD, D=D, xemb=xe, c_prev=c, h_out=ho, c_out=co, act_out=act),
                 part, cnt, gate_D=D)
    gts = x.double() @ Wx.double().T + h.double() @ Wh.double().T + xe.double()
    i_, f_, g_, o_ = _sig(gts[:, :D]), _sig(gts[:, D:2 * D]), torch.tanh(gts[:, 2 * D:3 * D]), _sig(gts[:, 3 * D:])
    c1 = f_ * c.double() + i_ * g_
    assert _rel(co, c1) < 2e-6 and _rel(ho, o_ * torch.tanh(c1)) < 2e-6
    assert _rel(act, torch.cat([i_, f_, g_, o_], 1)) < 2e-6
    # LSTM backward (rows >= bt zero)
    dg1, dgp1, dad1 = r(Bm, 4 * D), r(Bm, E), r(Bm, 32)
    Wb = r(D, 4 * D + E + 32) * 0.1
    dhd, dci, ccur = r(Bm, D), r(Bm, D), r(Bm, D)
    dgo, dco = torch.empty(Bm, 4 * D, device=DEV), torch.empty(Bm, D, device=DEV)
    bt = 61
    KB = 4 * D + E + 32
    K.dstep_gemm([(dg1, 4 * D, Wb, KB, 4 * D), (dgp1, E, Wb[:, 4 * D:], KB, E), (dad1, 32, Wb[:, 4 * D + E:], KB, 32)],
                 Bm, D, 16, S, dict(mode=CAPMI_DSTEP_LSTM_BWD, D=D, dhd=dhd, dc_in=dci, act=act, c_prev=c,
                                    c_cur=ccur, dgates=dgo, dc_out=dco, bt=bt), part, cnt)
    dh = torch.cat([dg1, dgp1, dad1], 1).double() @ Wb.double().T + dhd.double()
    a = act.double()
    ig, fg, cg, og = a[:, :D], a[:, D:2 * D], a[:, 2 * D:3 * D], a[:, 3 * D:]
    tc = torch.tanh(ccur.double())
    dc = dci.double() + dh * og * (1 - tc * tc)
    want = torch.cat([dc * cg * ig * (1 - ig), dc * c.double() * fg * (1 - fg), dc * ig * (1 - cg * cg),
                      dh * tc * og * (1 - og)], 1)
    want[bt:] = 0
    assert _rel(dgo, want) < 2e-6
    wdc = dc * fg
    wdc[bt:] = 0
    assert _rel(dco, wdc) < 2e-6
    # GATE_BWD
    dg, Wg = r(Bm, 4 * D), r(E, 4 * D) * 0.1
    gate, awe = torch.rand(Bm, E, generator=g).to(DEV), r(Bm, E)
    dawe, dgp = torch.empty(Bm, E, device=DEV), torch.empty(Bm, E, device=DEV)
    K.dstep_gemm([(dg, 4 * D, Wg, 4 * D, 4 * D)], Bm, E, 64, S,
                 dict(mode=CAPMI_DSTEP_GATE_BWD, gate=gate, awe=awe, dawe_out=dawe, dgp=dgp), part, cnt)
    d = dg.double() @ Wg.double().T
    gd = gate.double()
    assert _rel(dawe, d * gd) < 2e-6 and _rel(dgp, d * awe.double() * gd * (1 - gd)) < 2e-6
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0  # every last arriver reset its counter


def _step(monkeypatch, mode, cfg, enc, caps, lens, dup, with_denc):
    from capmi import decoder_fn as DF
    monkeypatch.setenv("CAPMI_DEC_FUSED", mode)
    dec, _ = make_decoder(cfg["A"], cfg["D"], cfg["M"], cfg["V"], cfg["seed"], DEV, emb_dtype=cfg.get("emb", np.float32))
    if cfg.get("ft_emb"):
        dec.fine_tune_embeddings(True)
    dec.train()
    grads = {n: torch.zeros_like(q) for n, q in dec.named_parameters() if q.requires_grad}
    denc = torch.empty_like(enc) if with_denc else None
    loss, preds, alphas = DF.fused_loss_and_grads(dec, enc, caps, lens, 1.0, grads, denc=denc, dup=dup)
    torch.cuda.synchronize()
    return loss, preds, alphas, grads, denc


@pytest.mark.parametrize("cfg", [
    dict(A=512, D=512, M=512, V=8100, B=64, L=25, ragged=True, seed=5, F=7, dup=2, denc=False),
    dict(A=512, D=512, M=768, V=600, B=64, L=25, ragged=False, seed=6, F=14, dup=1, denc=True),
    dict(A=32, D=32, M=300, V=50, B=3, L=6, ragged=True, seed=7, F=14, dup=1, denc=True, emb=np.float64,
         ft_emb=True),
    dict(A=64, D=64, M=16, V=90, B=70, L=9, ragged=True, seed=8, F=2, dup=7, denc=True),
])
@pytest.mark.parametrize("mode", ["1", "2"])
def test_fused_loop_matches_generic(monkeypatch, cfg, mode):
    """mode "1" (fused attention kernels on the generic GEMMs' partials) and mode "2" (also the
    last-arriver GEMMs) vs the five-launch path: the same arithmetic, fp32 order / contraction aside."""
    B, L, V, F = cfg["B"], cfg["L"], cfg["V"], cfg["F"]
    g = torch.Generator().manual_seed(cfg["seed"])
    enc = torch.rand(B, F * F, 2048, generator=g).to(DEV)
    if cfg["dup"] > 1:
        enc = enc.view(B, F, F, 2048)
    lens = sorted([int(v) for v in torch.randint(2, L + 1, (B,), generator=g)], reverse=True) if cfg["ragged"] else [L] * B
    lens[0] = L
    caps = t(gen.captions(cfg["seed"], B, L, V, lens), DEV)
    got = _step(monkeypatch, mode, cfg, enc, caps, lens, cfg["dup"], cfg["denc"])
    want = _step(monkeypatch, "0", cfg, enc, caps, lens, cfg["dup"], cfg["denc"])
    assert _rel(got[0], want[0]) < 2e-6, "loss"
    assert _rel(got[1], want[1]) < 2e-5, "predictions"
    assert _rel(got[2], want[2]) < 2e-5, "alphas"
    from test_gpu_decoder import KINK_ROWS, _grad_check
    kinks = set()
    for n in want[3]:
        if n in KINK_ROWS or n.endswith("full_att.bias"):  # ReLU score kinks / shift-invariant zero: a different att_dec rounding may flip a few (b, p, a)
            kinks |= _grad_check(got[3][n].cpu(), want[3][n].cpu(), n)
        else:
            assert _rel(got[3][n], want[3][n]) < 2e-5, n
    assert len(kinks) <= 2, kinks
    if cfg["denc"]:
        assert _rel(got[4], want[4]) < 2e-5, "d encoder_out"
    os.environ.pop("CAPMI_DEC_FUSED", None)
