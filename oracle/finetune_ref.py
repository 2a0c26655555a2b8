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
                        dfeat_only=False, masks=None, record=None, pre=None):
    """Returns dict(loss, feats, enc_raw, dec_raw, enc_new, dec_new, net) -- raw = unclamped
    gradients (what the GPU writes), new = parameters after clamp + Adam (one step).

    ``dtype=torch.float64`` runs the ENCODER in fp64 (the decoder keeps the reference's fp32
    LSTM input cast, Q6): the "exact" answer the fp32 paths are measured against, since
    train-mode BatchNorm at random init is ill-conditioned. ``masks`` / ``record`` / ``pre``: the
    encoder's trainable ReLUs on a given branch (encoder_backward_masked)."""
    net = build_resnet101(resnet_params).to(dtype)
    net.train()
    names = trainable_names(net)
    for n, q in net.named_parameters():
        q.requires_grad_(n in names)
    if masks is None and record is None and pre is None:
        feats = encoder_attention_forward(net, imgs.to(dtype))                # :389 encoder(imgs)
    else:
        feats = encoder_features_on_branch(net, imgs.to(dtype), masks, record, pre)
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


def _relu_at(z, name, masks, record, pre=None):
    """ReLU whose 0/1 mask is ``masks[name]`` when given (else z > 0); the mask taken is recorded.
    z * mask has the same value and the same gradient as torch.relu(z) under that mask
    (threshold_backward passes the gradient where z > 0)."""
    m = masks[name] if masks is not None else (z.detach() > 0)
    if record is not None:
        record[name] = m
    if pre is not None:
        pre[name] = z.detach().clone()
    return z * m.to(z.dtype)


def encoder_features_on_branch(net, imgs, masks=None, record=None, pre=None):
    """encoder_attention_forward (models/encoder.py:97-110) with the trainable blocks' ReLUs on a given
    branch (see encoder_backward_masked); masks/record/pre None: the plain forward."""
    x = net.maxpool(net.relu(net.bn1(net.conv1(imgs))))
    x = net.layer1(x)
    for li in (2, 3, 4):
        for bi, blk in enumerate(getattr(net, f"layer{li}")):
            tag = f"layer{li}.{bi}"
            idt = x if blk.downsample is None else blk.downsample(x)
            a1 = _relu_at(blk.bn1(blk.conv1(x)), tag + ".relu1", masks, record, pre)
            a2 = _relu_at(blk.bn2(blk.conv2(a1)), tag + ".relu2", masks, record, pre)
            x = _relu_at(blk.bn3(blk.conv3(a2)) + idt, tag + ".relu3", masks, record, pre)
    return torch.nn.functional.adaptive_avg_pool2d(x, (14, 14)).permute(0, 2, 3, 1)


def encoder_backward_masked(resnet_params, imgs, dfeat, dtype=torch.float64, layers=(3, 4, 23, 3), masks=None,
                            record=None, pre=None):
    """encoder_backward with the ReLUs of the trainable blocks (layer2-4: after bn1, after bn2, and the
    block output relu(bn3(y3) + identity), models/encoder.py:90-91 via torchvision's Bottleneck) taken
    on a GIVEN branch: ``masks[f"{layer}.{block}.relu{1,2,3}"]`` (bool, NCHW). ``record`` receives the
    masks this forward used (its own sign tests when ``masks`` is None), ``pre`` the pre-activations.

    Why: the encoder is piecewise linear in its ReLUs. An fp32 forward whose error is at rounding
    level still lands some pre-activation within that error of 0 on the other side of it, and each
    such flip moves the gradient by a full element of the upstream gradient -- a discrete event
    that no arithmetic tolerance describes. Differentiating the fp64 forward on the fp32 run's own
    branch compares the two on the same piecewise-linear function, where the gradient IS a
    continuous function of the arithmetic (the flips themselves are counted separately)."""
    net = build_resnet101(resnet_params, layers).to(dtype)
    net.train()
    names = trainable_names(net)
    for n, q in net.named_parameters():
        q.requires_grad_(n in names)
    feats = encoder_features_on_branch(net, imgs.to(dtype), masks, record, pre)
    feats.backward(dfeat.to(dtype))
    named = dict(net.named_parameters())
    return feats.detach(), {n: named[n].grad.detach().clone() for n in names}, net


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
