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
