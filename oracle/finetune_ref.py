"""ORACLE (test infrastructure): CPU restatement of one 'attention' training step with the
encoder fine-tuned (BASELINE config 4; models/attention.py:287-452 with --fine_tune_encoder,
models/encoder.py:112-121 fine_tune(True) -> layer2, layer3, layer4 trainable).

Composition of the two pinned restatements: oracle/resnet_ref.py (encoder, BatchNorm in train
mode because the reference calls encoder.train(), models/attention.py:374) and
oracle/decoder_ref.py (decoder, loss, clamp, Adam). torch-CPU autograd provides the backward.

Pinned by tests/golden/train_step_finetune.npz (the reference's own train() loop, with only the
Q9 defect patched: the reference builds its encoder optimizer over an all-frozen encoder).
Conv/BN arithmetic itself stays "parity unpinned" (torchvision is absent, see resnet_ref).
Never imported by the product.
"""
import torch

from . import decoder_ref as R
from .resnet_ref import build_resnet101, encoder_attention_forward

ENC_PREFIX = ("layer2.", "layer3.", "layer4.")


def trainable_names(net):
    """children()[5:] of the encoder's Sequential = layer2..layer4 (models/encoder.py:112-121)."""
    return [n for n, _ in net.named_parameters() if n.startswith(ENC_PREFIX)]


def finetune_train_step(resnet_params, dec_params, dec_trainable, imgs, captions, caption_lengths,
                        alpha_c=1.0, grad_clip=5.0, enc_lr=1e-4, dec_lr=1e-4, dtype=torch.float32,
                        dfeat_only=False):
    """Returns dict(loss, feats, enc_raw, dec_raw, enc_new, dec_new, net) -- raw = unclamped
    gradients (what the GPU writes), new = parameters after clamp + Adam (one step).

    ``dtype=torch.float64`` runs the ENCODER in fp64 (the decoder keeps the reference's fp32
    LSTM input cast, Q6): the "exact" answer the fp32 paths are measured against, since
    train-mode BatchNorm at random init is ill-conditioned."""
    net = build_resnet101(resnet_params).to(dtype)
    net.train()
    names = trainable_names(net)
    for n, q in net.named_parameters():
        q.requires_grad_(n in names)
    feats = encoder_attention_forward(net, imgs.to(dtype))                    # :389 encoder(imgs)
    leaves = {k: v.detach().clone().requires_grad_(k in dec_trainable) for k, v in dec_params.items()}
    preds, caps, dl, alphas = R.decoder_forward(leaves, feats.float() if dtype != torch.float32 else feats,
                                                captions, caption_lengths)    # :393
    loss = R.attention_loss(preds, caps, dl, alphas, alpha_c)                 # :401-414
    loss.backward()                                                           # :419
    named = dict(net.named_parameters())
    enc_raw = {n: named[n].grad.detach().clone() for n in names}
    dec_raw = {k: leaves[k].grad.detach().clone() for k in dec_trainable}
    enc_new, _ = R.adam_step({n: named[n].detach() for n in names}, R.clip_gradient(enc_raw, grad_clip), {},
                             lr=enc_lr)                                       # :422-430
    dec_new, _ = R.adam_step({k: dec_params[k] for k in dec_trainable}, R.clip_gradient(dec_raw, grad_clip), {},
                             lr=dec_lr)
    return dict(loss=loss.detach(), feats=feats.detach(), enc_raw=enc_raw, dec_raw=dec_raw, enc_new=enc_new,
                dec_new=dec_new, net=net)


def encoder_backward(resnet_params, imgs, dfeat, dtype=torch.float64, layers=(3, 4, 23, 3)):
    """Encoder-only: features and d(<features, dfeat>)/d(layer2-4 params) by autograd
    (``layers``: blocks per stage; shallower stacks are better conditioned in train-mode BN)."""
    net = build_resnet101(resnet_params, layers).to(dtype)
    net.train()
    names = trainable_names(net)
    for n, q in net.named_parameters():
        q.requires_grad_(n in names)
    feats = encoder_attention_forward(net, imgs.to(dtype))
    feats.backward(dfeat.to(dtype))
    named = dict(net.named_parameters())
    return feats.detach(), {n: named[n].grad.detach().clone() for n in names}, net
