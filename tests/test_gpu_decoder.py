"""GPU: the capmi attention decoder vs the CPU oracle and the reference's golden vectors.

Tolerances (BASELINE north_star): decoder logits rtol 1e-4, attention weights atol 1e-5.
Logit comparisons carry an absolute floor of 1e-5 (logits cross zero). Gradients are
checked at rtol 2e-3 with an absolute floor of 1e-3 * max|g| per tensor: the hoisted
weight gradients (one GEMM over all t instead of T summed per-step products) reorder
fp32 sums over up to B*P = 12544 terms."""
import numpy as np
import pytest
import torch

import gen
from helpers import assert_close, make_decoder, t
from oracle import decoder_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_RTOL, LOGIT_ATOL = 1e-4, 1e-5
ALPHA_ATOL = 1e-5


@pytest.mark.parametrize("tag", ["small_ragged", "small_full", "prod"])
def test_forward_matches_golden(golden, tag):
    fx = golden(f"decoder_forward_{tag}")
    m = fx["meta"]
    dec, _ = make_decoder(m["A"], m["D"], m["M"], m["V"], m["seed"], DEV)
    dec.eval()
    enc = t(gen.encoder_features(m["seed"], m["B"]), DEV)
    with torch.no_grad():
        preds, _, dl, alphas = dec(enc, t(fx["captions"], DEV), m["lengths"])
        h0, c0 = dec.init_hidden_state(enc.view(m["B"], -1, 2048))
    torch.cuda.synchronize()
    assert dl == m["decode_lengths"]
    assert_close(h0, t(fx["h0"]), 1e-5, 1e-6, "h0")
    assert_close(c0, t(fx["c0"]), 1e-5, 1e-6, "c0")
    assert_close(alphas, t(fx["alphas"]), 0.0, ALPHA_ATOL, "alphas")
    if "predictions" in fx:
        assert_close(preds, t(fx["predictions"]), LOGIT_RTOL, LOGIT_ATOL, "predictions")
    else:
        idx = fx["predictions__idx"]
        got = preds.reshape(-1).cpu()[torch.from_numpy(idx)]
        assert_close(got, t(fx["predictions__val"]), LOGIT_RTOL, LOGIT_ATOL, "predictions samples")


@pytest.mark.parametrize("tag", ["prod", "small"])
def test_soft_attention_matches_golden(golden, tag):
    from models.attention import SoftAttention
    fx = golden(f"soft_attention_{tag}")
    m = fx["meta"]
    B, P, E, D, A, s = m["B"], m["P"], m["E"], m["D"], m["A"], m["seed"]
    att = SoftAttention(E, D, A)
    sd = {"enc_att.weight": gen.uniform(s, "ea.w", (A, E), -E ** -.5, E ** -.5),
          "enc_att.bias": gen.uniform(s, "ea.b", (A,), -E ** -.5, E ** -.5),
          "dec_att.weight": gen.uniform(s, "da.w", (A, D), -D ** -.5, D ** -.5),
          "dec_att.bias": gen.uniform(s, "da.b", (A,), -D ** -.5, D ** -.5),
          "full_att.weight": gen.uniform(s, "fa.w", (1, A), -A ** -.5, A ** -.5),
          "full_att.bias": gen.uniform(s, "fa.b", (1,), -A ** -.5, A ** -.5)}
    att.load_state_dict({k: t(v) for k, v in sd.items()})
    att = att.to(DEV)
    with torch.no_grad():
        awe, alpha = att(t(gen.uniform(s, "enc", (B, P, E), 0, 1), DEV), t(gen.uniform(s, "h", (B, D), -1, 1), DEV))
    assert_close(alpha, t(fx["alpha"]), 0.0, ALPHA_ATOL, "alpha")
    assert_close(awe, t(fx["awe"]), 1e-4, 1e-5, "awe")


def _attention_ref64(enc, h, ps, off=None):
    """SoftAttention.forward (models/attention.py:43-61) in fp64 torch: the autograd reference (off: an
    optional (B, P) zero added to the scores, to read d(loss)/d(score))."""
    att = torch.relu(enc @ ps["ea.w"].T + ps["ea.b"] + (h @ ps["da.w"].T + ps["da.b"])[:, None, :])
    score = (att @ ps["fa.w"].T).squeeze(2) + ps["fa.b"]
    alpha = torch.softmax(score if off is None else score + off, dim=1)
    return (enc * alpha[:, :, None]).sum(1), alpha


def test_soft_attention_and_init_hidden_backward():
    """The standalone SoftAttention / init_hidden_state are differentiable (verdict r01 weak 10):
    every input and parameter gradient vs fp64 torch autograd, rtol 1e-4 + max(1e-5 * max|g|, 1e-6)."""
    from models.attention import SoftAttention
    g = torch.Generator().manual_seed(5)
    B, P, E, D, A = 3, 13, 64, 32, 48
    torch.manual_seed(5)  # the module's default init draws from the global generator: fix it
    att = SoftAttention(E, D, A).to(DEV)
    enc = torch.rand(B, P, E, generator=g)
    h = torch.rand(B, D, generator=g) * 2 - 1
    r1, r2 = torch.randn(B, E, generator=g), torch.randn(B, P, generator=g)
    e_d, h_d = enc.to(DEV).requires_grad_(), h.to(DEV).requires_grad_()
    awe, alpha = att(e_d, h_d)
    ((awe * r1.to(DEV)).sum() + (alpha * r2.to(DEV)).sum()).backward()
    names = {"ea": att.enc_att, "da": att.dec_att, "fa": att.full_att}
    ps = {f"{k}.{w}": getattr(m, "weight" if w == "w" else "bias").detach().cpu().double().requires_grad_()
          for k, m in names.items() for w in ("w", "b")}
    e64, h64 = enc.double().requires_grad_(), h.double().requires_grad_()
    a64, al64 = _attention_ref64(e64, h64, ps)
    ((a64 * r1.double()).sum() + (al64 * r2.double()).sum()).backward()
    torch.cuda.synchronize()

    # d full_att.bias = sum over the B*P scores of d(loss)/d(score), exactly 0 (softmax is shift-invariant):
    # an fp32 sum that cancels, so its tolerance is relative to the magnitude of the summed terms
    off = torch.zeros(B, P, dtype=torch.float64, requires_grad=True)
    a_o, al_o = _attention_ref64(enc.double(), h.double(), {k: v.detach() for k, v in ps.items()}, off)
    ((a_o * r1.double()).sum() + (al_o * r2.double()).sum()).backward()
    dscore_l1 = float(off.grad.abs().sum())

    def close(got, want, name, floor=1e-6):
        want = want.float()
        atol = max(1e-5 * float(want.abs().max()), floor)
        assert_close(got.detach().cpu().reshape(want.shape), want, 1e-4, atol, name)
    close(awe, a64.detach(), "awe")
    close(alpha, al64.detach(), "alpha")
    close(e_d.grad, e64.grad, "d enc")
    close(h_d.grad, h64.grad, "d h")
    for k, m in names.items():
        close(m.weight.grad, ps[f"{k}.w"].grad, f"d {k}.weight")
        close(m.bias.grad, ps[f"{k}.b"].grad, f"d {k}.bias", floor=1e-5 * dscore_l1 if k == "fa" else 1e-6)

    # init_hidden_state (:151-164) on the decoder's E = 2048 features
    dec, _ = make_decoder(A, D, 16, 40, 3, DEV)
    enc = torch.rand(B, P, 2048, generator=g)
    rh, rc = torch.randn(B, D, generator=g), torch.randn(B, D, generator=g)
    e_d = enc.to(DEV).requires_grad_()
    h0, c0 = dec.init_hidden_state(e_d)
    ((h0 * rh.to(DEV)).sum() + (c0 * rc.to(DEV)).sum()).backward()
    m64 = enc.double().requires_grad_()
    wl = {n: dict(dec.named_parameters())[n].detach().cpu().double().requires_grad_()
          for n in ("h_lin.weight", "h_lin.bias", "c_lin.weight", "c_lin.bias")}
    mean = m64.mean(1)
    h64 = mean @ wl["h_lin.weight"].T + wl["h_lin.bias"]
    c64 = mean @ wl["c_lin.weight"].T + wl["c_lin.bias"]
    ((h64 * rh.double()).sum() + (c64 * rc.double()).sum()).backward()
    torch.cuda.synchronize()
    close(e_d.grad, m64.grad, "init d enc")
    for n, w in wl.items():
        close(dict(dec.named_parameters())[n].grad, w.grad, f"init d {n}")


KINK_ROWS = ("attention.enc_att.weight", "attention.enc_att.bias", "attention.dec_att.weight",
             "attention.dec_att.bias")


def _grad_check(got, want, name):
    """Returns the set of rows excused by the ReLU-kink rule (empty for other parameters)."""
    if name.endswith("attention.full_att.bias"):
        # d loss / d b_full = sum_p dalpha-softmax-backward = 0 exactly (softmax is shift
        # invariant); the reference and capmi both return fp32 rounding noise here.
        assert float(got.abs().max()) < 1e-6 and float(want.abs().max()) < 1e-6, name
        return set()
    scale = float(want.abs().max()) if want.numel() else 1.0
    if name.split(" ")[-1] in KINK_ROWS:
        # The attention uses ReLU (models/attention.py:56). Where a pre-activation
        # att_enc + att_dec lands within fp32 rounding of 0, the GPU and the CPU reference can
        # take opposite sides of the kink: one such (b, p, a, t) changes d(att_enc)[b, p, a] and
        # d(att_dec)_t[b, a] by a full term, i.e. row a of dW_enc_att and of dW_dec_att. At most
        # 2 such rows are excused (a few flips are expected among B*P*A*T ~ 1e7
        # pre-activations), every other row must match, and the caller checks that the excused
        # rows of the two weights coincide (same a: the kink, not a kernel error).
        g2, w2 = got.reshape(got.shape[0], -1).double().cpu(), want.reshape(want.shape[0], -1).double()
        bad_rows = ((g2 - w2).abs() > 1e-3 * scale + 2e-3 * w2.abs() + 1e-9).any(1)
        assert int(bad_rows.sum()) <= 2, f"{name}: {int(bad_rows.sum())} rows out of tolerance"
        keep = ~bad_rows
        assert_close(g2[keep], w2[keep], 2e-3, 1e-3 * scale + 1e-9, name)
        return set(bad_rows.nonzero().view(-1).tolist())
    assert_close(got, want, 2e-3, 1e-3 * scale + 1e-9, name)
    return set()


@pytest.mark.parametrize("precision", ["fp32", "fp32-x3"])
@pytest.mark.parametrize("cfg", [
    dict(A=32, D=32, M=16, V=50, B=3, L=7, lengths=None, seed=41, emb=np.float32, ft_emb=False),
    dict(A=32, D=32, M=300, V=50, B=3, L=6, lengths=[6, 5, 3], seed=42, emb=np.float64, ft_emb=True),
    dict(A=512, D=512, M=512, V=8100, B=4, L=25, lengths=None, seed=43, emb=np.float32, ft_emb=False),
])
def test_fused_train_step_matches_oracle(cfg, precision):
    """capmi fused loss + BPTT + clamp/Adam vs the oracle's reference-restated step (fp32-x3: the
    decoder GEMMs as fp32-accurate three-term bf16 splits, same tolerances)."""
    from capmi import decoder_fn as DF
    from capmi.optim import Adam
    dec, p = make_decoder(cfg["A"], cfg["D"], cfg["M"], cfg["V"], cfg["seed"], DEV, emb_dtype=cfg["emb"])
    dec.set_compute_precision(precision)
    dec.fine_tune_embeddings(cfg["ft_emb"])
    dec.train()
    B, L, V = cfg["B"], cfg["L"], cfg["V"]
    enc = gen.encoder_features(cfg["seed"], B)
    caps = gen.captions(cfg["seed"], B, L, V, cfg["lengths"])
    lens = list(cfg["lengths"]) if cfg["lengths"] else [L] * B
    trainable = [n for n, q in dec.named_parameters() if q.requires_grad]
    opt = Adam([q for n, q in dec.named_parameters() if q.requires_grad], lr=1e-4)
    opt.set_clip(5.0)
    grads = {n: q.grad for n, q in dec.named_parameters() if q.requires_grad}
    loss, preds, alphas = DF.fused_loss_and_grads(dec, t(enc, DEV), t(caps, DEV), lens, 1.0, grads)
    torch.cuda.synchronize()
    ref = R.train_step(p, set(trainable), t(enc), t(caps), lens)
    rloss, rpreds, ralphas, rraw, _, rnew, _ = ref
    assert_close(loss.view(()), rloss, 1e-5, 1e-6, "loss")
    assert_close(preds, rpreds, LOGIT_RTOL, LOGIT_ATOL, "predictions")
    assert_close(alphas, ralphas, 0.0, ALPHA_ATOL, "alphas")
    excused = {n: _grad_check(grads[n].view_as(rraw[n]), rraw[n], "grad " + n) for n in trainable}
    kinks = set().union(*(excused.get(n, set()) for n in KINK_ROWS))
    assert len(kinks) <= 2 and excused.get("attention.dec_att.weight", set()) <= \
        excused.get("attention.enc_att.weight", set()) | excused.get("attention.enc_att.bias", set()), excused
    # clamp + Adam: the fused kernel vs the oracle's torch-Adam restatement fed the SAME
    # gradients (Adam's first step is ~lr*sign(g), so it is only well-conditioned this way)
    ours = {n: grads[n].detach().cpu().clone().view_as(rraw[n]) for n in trainable}
    want_p, _ = R.adam_step({n: p[n] for n in trainable}, R.clip_gradient(ours, 5.0), {}, lr=1e-4)
    opt.step()
    torch.cuda.synchronize()
    named = dict(dec.named_parameters())
    for n in trainable:
        assert_close(named[n].detach(), want_p[n], 1e-6, 1e-9, "adam step " + n)
    _ = rnew


@pytest.mark.parametrize("precision", ["fp32", "fp32-x3"])
@pytest.mark.parametrize("F,d,cfg", [
    (7, 2, dict(A=512, D=512, M=512, V=8100, B=4, L=25, seed=44)),  # 224x224: 7x7 -> 14x14
    (2, 7, dict(A=32, D=32, M=16, V=50, B=3, L=7, seed=45))])       # 64x64: 2x2 -> 14x14
def test_fused_dedup_matches_oracle(F, d, cfg, precision):
    """The decoder on the F*F distinct rows of pixel-duplicated features (dup = d) against the
    oracle run on the reference's pooled (F d) x (F d) map: loss, predictions, alphas over all
    positions and every gradient, under the rules of test_fused_train_step_matches_oracle."""
    from capmi import decoder_fn as DF
    dec, p = make_decoder(cfg["A"], cfg["D"], cfg["M"], cfg["V"], cfg["seed"], DEV)
    dec.set_compute_precision(precision)
    dec.train()
    B, L, V = cfg["B"], cfg["L"], cfg["V"]
    g = torch.Generator().manual_seed(cfg["seed"])
    distinct = torch.rand(B, F, F, 2048, generator=g)  # post-ReLU-like features
    pooled = distinct.repeat_interleave(d, 1).repeat_interleave(d, 2)  # AdaptiveAvgPool2d(F d) of F x F
    caps = gen.captions(cfg["seed"], B, L, V, None)
    trainable = [n for n, q in dec.named_parameters() if q.requires_grad]
    grads = {n: torch.zeros_like(q) for n, q in dec.named_parameters() if q.requires_grad}
    denc = torch.empty(B, F, F, 2048, device=DEV)  # d(loss)/d(F x F map), as the fine-tune step uses it
    loss, preds, alphas = DF.fused_loss_and_grads(dec, distinct.to(DEV), t(caps, DEV), [L] * B, 1.0, grads,
                                                  dup=d, denc=denc)
    torch.cuda.synchronize()
    assert tuple(alphas.shape) == (B, L - 1, (F * d) ** 2)
    rloss, rpreds, ralphas, rraw, _, _, _ = R.train_step(p, set(trainable), pooled.reshape(B, -1, 2048),
                                                         t(caps), [L] * B)
    assert_close(loss.view(()), rloss, 1e-5, 1e-6, "loss")
    assert_close(preds, rpreds, LOGIT_RTOL, LOGIT_ATOL, "predictions")
    assert_close(alphas, ralphas, 0.0, ALPHA_ATOL, "alphas")
    excused = {n: _grad_check(grads[n].view_as(rraw[n]), rraw[n], "grad " + n) for n in trainable}
    kinks = set().union(*(excused.get(n, set()) for n in KINK_ROWS))
    assert len(kinks) <= 2, excused
    # d(map): the reference's d(pooled features) summed over each d x d duplicate group
    pin = pooled.reshape(B, -1, 2048).clone().requires_grad_()
    pr, cp, dl, al = R.decoder_forward(dict(p), pin, t(caps), [L] * B)
    R.attention_loss(pr, cp, dl, al, 1.0).backward()
    want = pin.grad.view(B, F, d, F, d, 2048).sum((2, 4))
    assert_close(denc.cpu(), want, 2e-3, 1e-3 * float(want.abs().max()), "d map")


def test_dedup_kernels_exact():
    """capmi_att_alpha_expand / capmi_att_dup_pick against torch indexing (exact)."""
    from capmi import kernels as K
    F, d, B, T = 7, 2, 3, 5
    aq = torch.rand(B, T, F * F, device=DEV)
    ap = torch.empty(B, T, (F * d) ** 2, device=DEV)
    K.att_alpha_expand(aq, B * T, F, d, ap)
    want = aq.view(B, T, F, F).repeat_interleave(d, 2).repeat_interleave(d, 3).reshape(B, T, -1) / (d * d)
    torch.cuda.synchronize()
    assert torch.equal(ap, want)
    full = torch.rand(B, (F * d) ** 2, device=DEV)
    out = torch.empty(B, F * F, device=DEV)
    K.att_dup_pick(full, B, F, d, out)
    torch.cuda.synchronize()
    assert torch.equal(out, full.view(B, F * d, F * d)[:, ::d, ::d].reshape(B, -1))


def test_autograd_path_reference_loss():
    """The reference's own loss code (pack_padded_sequence + CrossEntropyLoss + reg) on top of
    capmi's differentiable forward: gradients reach the parameters through AttentionDecoderFn."""
    from torch.nn.utils.rnn import pack_padded_sequence
    A, D, M, V, B, L, seed = 32, 32, 16, 50, 3, 6, 44
    dec, p = make_decoder(A, D, M, V, seed, DEV)
    dec.train()
    enc = gen.encoder_features(seed, B)
    caps = gen.captions(seed, B, L, V, [6, 4, 3])
    lens = [6, 4, 3]  # ragged, sorted: exercises batch_size_t
    preds, caps_s, dl, alphas = dec(t(enc, DEV), t(caps, DEV), lens)
    targets = caps_s[:, 1:]
    scores = pack_padded_sequence(preds, dl, batch_first=True).data
    tg = pack_padded_sequence(targets, dl, batch_first=True).data
    loss = torch.nn.CrossEntropyLoss()(scores, tg) + ((1.0 - alphas.sum(dim=1)) ** 2).mean()
    loss.backward()
    trainable = [n for n, q in dec.named_parameters() if q.requires_grad]
    ref = R.train_step(p, set(trainable), t(enc), t(caps), lens)
    assert_close(loss.detach(), ref[0], 1e-5, 1e-6, "loss")
    named = dict(dec.named_parameters())
    for n in trainable:
        _grad_check(named[n].grad, ref[3][n], "grad " + n)


def test_dropout_mask_replay():
    """Dropout (p=0.5, train mode): replaying capmi's mask through the oracle gives the same logits."""
    from capmi import kernels as K
    A, D, M, V, B, L, seed = 32, 32, 16, 50, 4, 8, 45
    dec, p = make_decoder(A, D, M, V, seed, DEV, dropout=0.5)
    dec.train()
    enc = gen.encoder_features(seed, B)
    caps = gen.captions(seed, B, L, V)
    torch.manual_seed(3)
    with torch.no_grad():
        preds, _, _, _ = dec(t(enc, DEV), t(caps, DEV), [L] * B)
    torch.manual_seed(3)
    s = int(torch.randint(0, 2 ** 62, (1,)).item())
    T = L - 1
    ones = torch.ones(T, B, D, device=DEV)
    mask = torch.empty_like(ones)
    K.dropout(ones, ones.numel(), 0.5, s, mask)
    keep = (mask > 0).float().mean().item()
    assert 0.4 < keep < 0.6
    with torch.no_grad():
        rp, _, _, _ = R.decoder_forward(p, t(enc), t(caps), [L] * B, dropout_masks=mask.cpu())
    assert_close(preds, rp, LOGIT_RTOL, LOGIT_ATOL, "dropout predictions")
