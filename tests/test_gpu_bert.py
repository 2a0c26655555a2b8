"""GPU: the 'bert_attention' variant (use_bert, models/attention.py:96-100,166-215,242-244;
BASELINE config 5) -- the decoder consumes precomputed (B, L+1, 768) word-level features
instead of its embedding table, and no gradient reaches the table.

bert-base-uncased cannot be fetched offline, so the features come from
capmi.data.SyntheticBertEmbedder; the oracle (oracle/decoder_ref.py with ``embeddings=``, the
reference's BERT branch) consumes the same tensor. Tolerances as tests/test_gpu_decoder.py:
logits rtol 1e-4 (+1e-5 floor), alphas atol 1e-5, gradients rtol 2e-3 with a 1e-3*max|g| floor."""
import pytest
import torch

import gen
from helpers import assert_close, t
from oracle import decoder_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bert_decoder(A, D, V, seed):
    from capmi.data import SyntheticBertEmbedder
    from models.attention import AttentionDecoder, AttentionDecoderParams
    from vocabulary import synthetic_vocab
    M = 768
    prm = AttentionDecoderParams()
    prm.attention_dim, prm.decoder_dim, prm.embed_size, prm.dropout = A, D, M, 0.0
    prm.vocab = synthetic_vocab(V)
    prm.use_bert = True
    dec = AttentionDecoder(DEV, prm)
    p = gen.decoder_params(seed, A, D, M, V)
    sd = dec.state_dict()
    for k, v in p.items():
        sd[k] = t(v).clone()
    dec.load_state_dict(sd)
    dec = dec.to(DEV)
    dec.bert_embedder = SyntheticBertEmbedder(V, M, device=DEV)
    return dec, {k: t(v) for k, v in p.items()}


@pytest.mark.parametrize("A,D,V,B,L", [(32, 32, 50, 3, 7), (512, 512, 8100, 2, 25)])
def test_bert_variant_train_step_matches_oracle(A, D, V, B, L):
    from capmi import decoder_fn as DF
    seed = 55
    dec, p = _bert_decoder(A, D, V, seed)
    dec.train()
    enc = gen.encoder_features(seed, B)
    caps = gen.captions(seed, B, L, V)
    emb = dec.bert_embedder(t(caps, DEV))
    assert tuple(emb.shape) == (B, L + 1, 768)
    named = dict(dec.named_parameters())
    grads = {n: torch.zeros_like(q) for n, q in named.items() if q.requires_grad}
    loss, preds, alphas = DF.fused_loss_and_grads(dec, t(enc, DEV), t(caps, DEV), [L] * B, 1.0, grads)
    torch.cuda.synchronize()
    trainable = {n for n in named if n != "embedding.weight"}
    leaves = {k: v.detach().clone().requires_grad_(k in trainable) for k, v in p.items()}
    rp, caps_s, dl, ra = R.decoder_forward(leaves, t(enc), t(caps), [L] * B, embeddings=emb.cpu())
    rl = R.attention_loss(rp, caps_s, dl, ra)
    rl.backward()
    assert_close(loss.view(()), rl.detach(), 1e-5, 1e-6, "loss")
    assert_close(preds, rp.detach(), 1e-4, 1e-5, "predictions")
    assert_close(alphas, ra.detach(), 0.0, 1e-5, "alphas")
    from test_gpu_decoder import KINK_ROWS, _grad_check  # ReLU-kink rows, zero full_att.bias rule
    excused = {n: _grad_check(grads[n].view_as(leaves[n].grad), leaves[n].grad, "grad " + n) for n in trainable}
    kinks = set().union(*(excused.get(n, set()) for n in KINK_ROWS))
    assert len(kinks) <= 2 and excused.get("attention.dec_att.weight", set()) <= \
        excused.get("attention.enc_att.weight", set()) | excused.get("attention.enc_att.bias", set()), excused
    assert float(grads["embedding.weight"].abs().max()) == 0.0  # frozen features: no table gradient


def test_bert_variant_autograd_surface():
    """decoder(enc, caps, lens) under autograd: the table gets no .grad (reference: BERT features
    are computed under no_grad, so Adam skips the embedding parameter)."""
    seed = 56
    dec, p = _bert_decoder(32, 32, 50, seed)
    dec.train()
    B, L = 2, 6
    enc = t(gen.encoder_features(seed, B), DEV)
    caps = t(gen.captions(seed, B, L, 50), DEV)
    preds, _, dl, alphas = dec(enc, caps, [L] * B)
    (preds.sum() + alphas.sum()).backward()
    torch.cuda.synchronize()
    assert dec.embedding.weight.grad is None
    assert dec.fc.weight.grad is not None and dec.decode_step.weight_ih.shape[1] == 768 + 2048
    with pytest.raises(RuntimeError):
        dec.bert_embedder = None
        dec(enc, caps, [L] * B)
