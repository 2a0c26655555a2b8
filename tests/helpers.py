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
