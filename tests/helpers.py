"""Shared builders for the parity tests (test infrastructure)."""
import numpy as np
import torch

import gen


def t(x, device="cpu"):
    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


def make_decoder(A, D, M, V, seed, device, emb_dtype=np.float32, dropout=0.0):
    """capmi AttentionDecoder with the seeded golden weights (gen.decoder_params)."""
    from models.attention import AttentionDecoder, AttentionDecoderParams
    from vocabulary import synthetic_vocab
    prm = AttentionDecoderParams()
    prm.attention_dim, prm.decoder_dim, prm.embed_size = A, D, M
    prm.dropout = dropout
    prm.vocab = synthetic_vocab(V)
    dec = AttentionDecoder(device, prm)
    p = gen.decoder_params(seed, A, D, M, V, emb_dtype=emb_dtype)
    if emb_dtype == np.float64:
        dec.load_pretrained_embeddins(t(p["embedding.weight"]).clone())
    sd = dec.state_dict()
    for k, v in p.items():
        sd[k] = t(v).clone()
    dec.load_state_dict(sd)
    return dec.to(device), {k: t(v) for k, v in p.items()}


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def ft_relu_masks(ft):
    """The ReLU branch a capmi fine-tune forward took in every trainable block (FineTuneRunner.state,
    read after forward, before backward), keyed as oracle.finetune_ref.encoder_backward_masked
    expects: relu1 / relu2 = [fma(y, scale, shift) > 0] (the sign of the exact value, which fp64
    y*s + b preserves; the backward kernels' own mask), relu3 = [out > 0] of the saved block output."""
    masks = {}
    N = ft.state["N"]
    for b in ft.state["blocks"]:
        H, W, H2, W2, wd, Co = b["H"], b["W"], b["H2"], b["W2"], b["wd"], b["Cout"]

        def nchw(x, h, w, c):
            return x[: N * h * w * c].view(N, h, w, c).permute(0, 3, 1, 2).double().cpu()

        (s1, b1, _), (s2, b2, _) = b["ss"][0], b["ss"][1]
        v = lambda a: a.detach().double().cpu().view(1, -1, 1, 1)  # noqa: E731
        masks[b["tag"] + ".relu1"] = nchw(b["y1"], H, W, wd) * v(s1) + v(b1) > 0
        masks[b["tag"] + ".relu2"] = nchw(b["y2"], H2, W2, wd) * v(s2) + v(b2) > 0
        masks[b["tag"] + ".relu3"] = nchw(b["out"], H2, W2, Co) > 0
    return masks


def decoder_att_masks(dup=1):
    """The attention-score ReLU decisions of the last capmi decoder forward, (T, B, P, A) bool over the
    reference's P positions: the score kernel takes relu(ATT_ENC[b, q] + AD[t, b]) in fp32 (att_enc and
    att_dec with their biases, both kept for the backward), whose sign the exact fp64 sum preserves.
    dup > 1: the distinct rows q of an F x F map, expanded to the pooled (F dup)^2 positions."""
    from capmi import decoder_fn as DF
    ws = next(iter(DF.CORE._ws.values()))
    ae, ad = ws.ATT_ENC.double().cpu(), ws.AD.double().cpu()
    T, B, A = ad.shape
    out = []
    for t_ in range(T):
        m = ae + ad[t_].unsqueeze(1) > 0  # (B, Q, A)
        if dup > 1:
            F_ = int(round(m.shape[1] ** 0.5))
            m = m.view(B, F_, F_, A).repeat_interleave(dup, 1).repeat_interleave(dup, 2).reshape(B, -1, A)
        out.append(m)
    return torch.stack(out)


def _oracle_att_preacts(p, enc, caps, lengths, dtype):
    """Per decode step of the oracle forward (oracle.decoder_ref.decoder_forward, models/attention.py:
    218-284) in ``dtype`` on its OWN attention-ReLU branch: yields (z, s) with z = the score pre-activation
    att_enc + att_dec (B, P, A) and s = its magnitude bound |enc| |W_ea|^T + |b_ea| + |h| |W_da|^T + |b_da|
    (the scale of the rounding error of the two dot products that form z). The attention-score ReLU is the
    decoder's only branch; its decisions at |z| within rounding of 0 differ between fp32 paths."""
    import torch.nn.functional as F
    from oracle import decoder_ref as R
    q = {k: v.to(dtype) for k, v in p.items()}
    e = enc.to(dtype).reshape(enc.shape[0], -1, enc.shape[-1])  # (B, P, D), as forward() flattens it (:231)
    emb = F.embedding(caps, q["embedding.weight"]).to(dtype)
    h, c = R.init_hidden_state(q, e)
    ae = R._lin(e, q, "attention.enc_att")  # loop-invariant (models/attention.py:54, recomputed there)
    sa = e.abs() @ q["attention.enc_att.weight"].abs().t() + q["attention.enc_att.bias"].abs()
    for t_ in range(max(lengths) - 1):
        ad = R._lin(h, q, "attention.dec_att")
        sd = h.abs() @ q["attention.dec_att.weight"].abs().t() + q["attention.dec_att.bias"].abs()
        z = ae + ad.unsqueeze(1)
        yield z, sa + sd.unsqueeze(1)
        att = R._lin(torch.relu(z), q, "attention.full_att").squeeze(2)
        alpha = torch.softmax(att, dim=1)
        awe = torch.sigmoid(R._lin(h, q, "f_beta")) * (e * alpha.unsqueeze(2)).sum(dim=1)
        h, c = R.lstm_cell(torch.cat([emb[:, t_, :], awe], 1), h, c, q)


def decoder_att_flips(p, enc, caps, lengths, dup=1):
    """The attention-score pre-activations z of the last capmi decoder forward (ATT_ENC + AD, kept for its
    backward; decoder_att_masks' source) against the fp64 oracle on its OWN branch, beside the fp32 CPU
    oracle's. Returns dict: n_gpu / n_cpu = ReLU decisions differing from fp64's (over the reference's P
    positions); err_gpu / err_cpu = rms(z - z64) / rms(z64); worst_gpu / worst_cpu = the largest flipped |z64|
    in fp32 unit roundoffs (2^-24) of z's magnitude bound s64 (a rounding-level decision sits within a few
    tens of them: the dot products have K = 2048 and 512)."""
    from capmi import decoder_fn as DF
    ws = next(iter(DF.CORE._ws.values()))
    ae_g, ad_g = ws.ATT_ENC.double().cpu(), ws.AD.double().cpu()
    u = 2.0 ** -24
    r = dict(n_gpu=0, n_cpu=0, worst_gpu=0.0, worst_cpu=0.0)
    e2 = {"gpu": 0.0, "cpu": 0.0}
    ref2 = 0.0
    for t_, ((z64, s64), (z32, _)) in enumerate(zip(_oracle_att_preacts(p, enc, caps, lengths, torch.float64),
                                                    _oracle_att_preacts(p, enc, caps, lengths, torch.float32))):
        zg = ae_g + ad_g[t_].unsqueeze(1)  # (B, Q, A)
        if dup > 1:
            B_, Q_, A_ = zg.shape
            F_ = int(round(Q_ ** 0.5))
            zg = zg.view(B_, F_, F_, A_).repeat_interleave(dup, 1).repeat_interleave(dup, 2).reshape(B_, -1, A_)
        ref2 += float((z64 ** 2).sum())
        for name, z in (("gpu", zg), ("cpu", z32.double())):
            e2[name] += float(((z - z64) ** 2).sum())
            bad = (z > 0) != (z64 > 0)
            n = int(bad.sum())
            if n:
                r["n_" + name] += n
                r["worst_" + name] = max(r["worst_" + name], float((z64[bad].abs() / (s64[bad] * u)).max()))
    r["err_gpu"], r["err_cpu"] = (e2["gpu"] / ref2) ** 0.5, (e2["cpu"] / ref2) ** 0.5
    return r


def mask_flips(got, ref):
    """Number of elements where two ReLU branches disagree, over all masks."""
    return sum(int((got[k] != ref[k]).sum()) for k in ref)


def assert_close(a, b, rtol, atol, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    diff = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = diff > tol
    if bad.any():
        i = int(torch.argmax((diff - tol).reshape(-1)))
        raise AssertionError(f"{what}: {int(bad.sum())}/{bad.numel()} elements out of tolerance "
                             f"(rtol {rtol}, atol {atol}); worst at {i}: got {a.reshape(-1)[i]:.8g} "
                             f"want {b.reshape(-1)[i]:.8g}; max abs diff {float(diff.max()):.3g}")
