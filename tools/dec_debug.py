"""Decoder backward diagnostics (GPU): re-derive the hoisted weight gradients in fp64 from the
GPU's own saved per-step buffers, to separate GEMM errors from upstream (BPTT) errors."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "image-captioning-with-different-decoders_amd"), REPO, os.path.join(REPO, "tests"),
          os.path.join(REPO, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen  # noqa: E402
from helpers import make_decoder, t  # noqa: E402


def main():
    from capmi import decoder_fn as DF
    DEV = "cuda"
    A = D = M = 512
    V, B, L, seed = 8100, 4, 25, 43
    dec, p = make_decoder(A, D, M, V, seed, DEV, emb_dtype=np.float32)
    dec.fine_tune_embeddings(False)
    dec.train()
    enc = gen.encoder_features(seed, B)
    caps = gen.captions(seed, B, L, V, None)
    grads = {n: torch.zeros_like(q) for n, q in dec.named_parameters() if q.requires_grad}
    loss, preds, alphas = DF.fused_loss_and_grads(dec, t(enc, DEV), t(caps, DEV), [L] * B, 1.0, grads)
    torch.cuda.synchronize()
    ws = DF.CORE._ws[next(iter(DF.CORE._ws))]
    T, P, E = L - 1, 196, 2048
    encd = t(enc, DEV).reshape(B * P, E).double()
    datt = ws.DATT.reshape(B * P, A).double()
    g = grads["attention.enc_att.weight"].double()
    ref = datt.T @ encd
    scale = (datt.abs().T @ encd.abs())
    err = (g - ref).abs()
    print("enc_att dW: max |g|", float(ref.abs().max()), "max err", float(err.max()),
          "max err/sum|ab|", float((err / (scale + 1e-30)).max()))
    bad = (err > 4e-6 * scale + 1e-12).nonzero()
    print("elements over 4e-6*sum|ab|:", bad.shape[0], bad[:10].tolist())
    # W_ih / fc weight grads from the saved buffers
    TB = T * B
    dg = ws.DG.reshape(TB, 4 * D).double()
    X = ws.X.reshape(TB, -1).double()
    gi = grads["decode_step.weight_ih"].double()
    r = dg.T @ X
    print("W_ih dW max err", float((gi - r).abs().max()), "max", float(r.abs().max()))


if __name__ == "__main__":
    main()
