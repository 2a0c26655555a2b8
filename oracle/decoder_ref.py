"""ORACLE (test infrastructure): CPU fp32 restatement of the reference's
attention-decoder training step, op for op (unhoisted ``enc_att``, ReLU
attention, fp64 round-trip on the LSTM input, CE over packed rows *with*
pads, doubly-stochastic regulariser, element-wise clamp, Adam).

Pinned against tests/golden/*.npz, which ``tests/golden/make_golden.py``
produced by running the real reference code (models/attention.py,
train_utils.py) in the survey container. Never imported by the product.
"""
import math

import torch
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence


def _lin(x, p, name):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def soft_attention(p, encoder_out, decoder_hidden, prefix="attention.", mask=None):
    """models/attention.py:43-61. ``mask`` (B, P, A bool, optional): take the score ReLU on that branch
    (z * mask: torch.relu's value and gradient when mask = z > 0) -- the GPU run's own decisions, so a
    pre-activation within rounding of 0 compares on the same piecewise-linear function."""
    att_enc = _lin(encoder_out, p, prefix + "enc_att")                     # :54
    att_dec = _lin(decoder_hidden, p, prefix + "dec_att")                  # :55
    z = att_enc + att_dec.unsqueeze(1)
    act = torch.relu(z) if mask is None else z * mask.to(z.dtype)
    att = _lin(act, p, prefix + "full_att").squeeze(2)                     # :56-57 (ReLU, not tanh)
    alpha = torch.softmax(att, dim=1)                                      # :58
    awe = (encoder_out * alpha.unsqueeze(2)).sum(dim=1)                   # :59-60
    return awe, alpha


def init_hidden_state(p, encoder_out):
    """models/attention.py:151-164."""
    mean_enc = encoder_out.mean(dim=1)
    return _lin(mean_enc, p, "h_lin"), _lin(mean_enc, p, "c_lin")


def lstm_cell(x, h, c, p):
    """nn.LSTMCell (models/attention.py:108-109): gates i, f, g, o."""
    gates = F.linear(x, p["decode_step.weight_ih"], p["decode_step.bias_ih"]) + \
        F.linear(h, p["decode_step.weight_hh"], p["decode_step.bias_hh"])
    i, f, g, o = gates.chunk(4, 1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(c2), c2


def decoder_forward(p, encoder_out, encoded_captions, caption_lengths, dropout_p=0.0,
                    dropout_masks=None, embeddings=None, att_masks=None):
    """models/attention.py:218-284 (regular-embedding branch, :247; ``embeddings`` (B, L', M)
    given = the BERT branch, :242-244, which uses precomputed features instead of the table).

    ``dropout_masks`` (optional, (T,B,D) of 0/1/(1-p) scale) replaces the
    reference's RNG-driven nn.Dropout so a GPU run's mask can be replayed; ``att_masks`` (optional,
    (T, B, P, A) bool) the attention-score ReLU decisions (soft_attention's ``mask``) per step."""
    B = encoder_out.size(0)
    E = encoder_out.size(-1)
    enc = encoder_out.reshape(B, -1, E)                                    # :230
    P = enc.size(1)
    decode_lengths = [l - 1 for l in caption_lengths]                      # :236-237
    T = max(decode_lengths)
    if embeddings is None:
        embeddings = F.embedding(encoded_captions, p["embedding.weight"])  # :247
    h, c = init_hidden_state(p, enc)                                       # :250
    V = p["fc.weight"].shape[0]
    wdt = p["decode_step.weight_ih"].dtype  # fp32 as in the reference; fp64 only for diagnostics
    predictions = torch.zeros(B, T, V, dtype=wdt)                          # :253-254
    alphas = torch.zeros(B, T, P, dtype=wdt)                               # :257-258
    for t in range(T):                                                     # :260
        bt = sum(l > t for l in decode_lengths)                            # :261
        awe, alpha = soft_attention(p, enc[:bt], h[:bt],
                                    mask=None if att_masks is None else att_masks[t, :bt])  # :267-268
        gate = torch.sigmoid(_lin(h[:bt], p, "f_beta"))                    # :270
        awe = gate * awe                                                   # :271
        x = torch.cat([embeddings[:bt, t, :].double(), awe.double()], 1)   # :274-275
        h, c = lstm_cell(x.to(wdt), h[:bt].to(wdt), c[:bt].to(wdt), p)     # :277-278 (.float())
        hd = h
        if dropout_masks is not None:
            hd = h * dropout_masks[t, :bt]
        elif dropout_p > 0:
            hd = F.dropout(h, dropout_p, True)
        predictions[:bt, t, :] = _lin(hd, p, "fc")                         # :279-280
        alphas[:bt, t, :] = alpha                                          # :281
    return predictions, encoded_captions, decode_lengths, alphas


def attention_loss(predictions, captions, decode_lengths, alphas, alpha_c=1.0):
    """models/attention.py:401-414: CE over pack_padded rows (no ignore_index,
    so pad positions are scored, Q2) + ((alpha_c - sum_t alpha)^2).mean()."""
    targets = captions[:, 1:]
    scores = pack_padded_sequence(predictions, decode_lengths, batch_first=True).data
    targets = pack_padded_sequence(targets, decode_lengths, batch_first=True).data
    loss = F.cross_entropy(scores, targets)
    return loss + ((alpha_c - alphas.sum(dim=1)) ** 2).mean()


def clip_gradient(grads, grad_clip):
    """train_utils.py:2-12: element-wise clamp_(-c, c) of every gradient."""
    return {k: g.clamp(-grad_clip, grad_clip) for k, g in grads.items()}


def adam_step(params, grads, state, lr=1e-4, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam (single-tensor CPU path, no weight decay, no amsgrad)
    as used at models/attention.py:352-355,428. Returns new params, state."""
    b1, b2 = betas
    new_p, new_s = {}, {}
    for k, p in params.items():
        g = grads[k]
        st = state.get(k)
        if st is None:
            st = {"step": 0, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
        step = st["step"] + 1
        m = st["exp_avg"].lerp(g, 1 - b1)
        v = st["exp_avg_sq"].mul(b2).addcmul(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        new_p[k] = p.addcdiv(m, denom, value=-(lr / bc1))
        new_s[k] = {"step": step, "exp_avg": m, "exp_avg_sq": v}
    return new_p, new_s


def train_step(p, trainable, encoder_out, captions, caption_lengths, alpha_c=1.0,
               grad_clip=5.0, lr=1e-4, state=None, dropout_masks=None, embeddings=None, att_masks=None):
    """One decoder step of models/attention.py:386-430 (dropout off unless
    masks are given). ``p``: dict of float tensors; ``trainable``: names that
    require grad (the reference's filter(requires_grad), :352-355).
    Returns (loss, predictions, alphas, grads(clamped), new_params, state)."""
    leaves = {k: (v.detach().clone().requires_grad_(k in trainable)) for k, v in p.items()}
    preds, caps, dl, alphas = decoder_forward(leaves, encoder_out, captions, caption_lengths,
                                              dropout_masks=dropout_masks, embeddings=embeddings,
                                              att_masks=att_masks)
    loss = attention_loss(preds, caps, dl, alphas, alpha_c)
    loss.backward()
    raw = {k: leaves[k].grad.detach().clone() for k in trainable}
    grads = clip_gradient(raw, grad_clip)
    new_p, new_s = adam_step({k: p[k] for k in trainable}, grads, state or {}, lr=lr)
    return loss.detach(), preds.detach(), alphas.detach(), raw, grads, new_p, new_s


# --------------------------------------------------------------------------
# Baseline decoder (config 1 surface), models/baseline.py:24-111,194-195
# --------------------------------------------------------------------------

def baseline_forward(p, img_features, captions):
    """models/baseline.py:81-111: prepend the image feature, LSTM, Linear."""
    caps = captions[:, :-1]
    emb = F.embedding(caps, p["embedding.weight"])
    x = torch.cat((img_features.unsqueeze(1).float(), emb.float()), 1)
    B, L, _ = x.shape
    H = p["lstm.weight_hh_l0"].shape[1]
    h = torch.zeros(B, H)
    c = torch.zeros(B, H)
    outs = []
    w = {"decode_step.weight_ih": p["lstm.weight_ih_l0"], "decode_step.weight_hh": p["lstm.weight_hh_l0"],
         "decode_step.bias_ih": p["lstm.bias_ih_l0"], "decode_step.bias_hh": p["lstm.bias_hh_l0"]}
    for t in range(L):
        h, c = lstm_cell(x[:, t], h, c, w)
        outs.append(h)
    return F.linear(torch.stack(outs, 1), p["linear.weight"], p["linear.bias"])


def baseline_loss(scores, captions, pad_idx=0):
    """models/baseline.py:194-195,224-225: CE with ignore_index=PAD against the
    captions *including* <start> (the reference's own alignment)."""
    return F.cross_entropy(scores.reshape(-1, scores.shape[2]), captions.reshape(-1),
                           ignore_index=pad_idx)
