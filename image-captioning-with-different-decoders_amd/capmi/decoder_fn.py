"""Autograd entry points and fused loss for the attention decoder.

* ``AttentionDecoderFn``: the differentiable ``AttentionDecoder.forward`` the
  reference's own training loop calls (models/attention.py:396): returns
  (predictions, alphas); its backward runs the capmi BPTT kernels.
* ``fused_loss_and_grads``: the whole loss of models/attention.py:401-414 (CE
  over the packed rows incl. pads + the doubly-stochastic regulariser) and the
  full decoder backward in one go, writing parameter gradients straight into the
  optimizer's flat buffer -- what capmi's own ``train()`` and bench.py run.
* ``soft_attention_forward`` / ``init_hidden_forward``: inference-only kernels
  for the standalone sub-modules (beam search uses them, gen_captions.py:62-72).
"""
import torch

from . import kernels as K
from ._lib import CAPMI_A_KMAJOR, CAPMI_B_NMAJOR_W
from .decoder_core import PNAMES, DecoderCore

CORE = DecoderCore()
_GEN = [0]


def decoder_params(dec):
    sd = dict(dec.named_parameters())
    p = {n: sd[n] for n in PNAMES}
    p["attention.full_att.weight"] = p["attention.full_att.weight"].view(-1)
    return p


def _prep_inputs(dec, encoder_out, encoded_captions):
    if not encoder_out.is_cuda:
        raise RuntimeError("capmi AttentionDecoder runs on the MI355X (HIP tensors only)")
    B = encoder_out.size(0)
    E = encoder_out.size(-1)
    enc = encoder_out.reshape(B, -1, E)
    if enc.dtype != torch.float32:
        raise TypeError("encoder_out must be float32")
    enc = enc.contiguous()
    caps = encoded_captions.to(device=enc.device, dtype=torch.int64).contiguous()
    return enc, caps


def dense_embeddings(dec, caps):
    """The BERT variant (use_bert, models/attention.py:166-215,242-244): (B, L+1, 768) word-level
    features from the decoder's ``bert_embedder`` (frozen, computed without grad), else None."""
    if not getattr(dec, "use_bert", False):
        return None
    with torch.no_grad():
        e = dec.bert_embeddings(caps)
    if e.dtype != torch.float32 or not e.is_cuda:
        raise TypeError("BERT embeddings must be float32 device tensors")
    return e.contiguous()


def _seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class AttentionDecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dec, enc, caps, decode_lengths, *params):
        p = dict(zip(PNAMES, params))
        p["attention.full_att.weight"] = p["attention.full_att.weight"].view(-1)
        drop = dec.dropout.p if dec.training else 0.0
        preds, alphas, st = CORE.forward(p, enc, caps, decode_lengths, dropout_p=drop,
                                         training=dec.training, seed=_seed() if drop > 0 else 0,
                                         emb_dense=dense_embeddings(dec, caps))
        _GEN[0] += 1
        st["gen"] = _GEN[0]
        ctx.st, ctx.p = st, p
        ctx.need = [n for n, t in zip(PNAMES, params) if t.requires_grad]
        ctx.enc_grad = enc.requires_grad
        return preds, alphas

    @staticmethod
    def backward(ctx, dpred, dalphas):
        st = ctx.st
        if st["gen"] != _GEN[0]:
            raise RuntimeError("capmi decoder: another forward of the same shape ran before this "
                               "backward and overwrote its saved per-step state")
        # the BERT variant's embeddings are frozen features: the (unused) table gets no gradient
        grads = {n: torch.empty_like(ctx.p[n]) for n in ctx.need
                 if not (st["dense_emb"] and n == "embedding.weight")}
        if dpred is None:
            dpred = torch.zeros(st["dm"].B, st["dm"].T, st["dm"].V, device=st["enc"].device)
        denc = torch.empty_like(st["enc"]) if ctx.enc_grad else None
        CORE.backward(ctx.p, st, grads, dpred.contiguous(), dalphas=None if dalphas is None else dalphas.contiguous(),
                      denc=denc)
        out = [None, denc, None, None]
        for n in PNAMES:
            g = grads.get(n)
            if g is not None and n == "attention.full_att.weight":
                g = g.view(1, -1)
            out.append(g)
        return tuple(out)


def decoder_forward(dec, encoder_out, encoded_captions, caption_lengths):
    """models/attention.py:218-284 on the capmi kernels."""
    enc, caps = _prep_inputs(dec, encoder_out, encoded_captions)
    decode_lengths = [int(l) - 1 for l in caption_lengths]
    params = [dict(dec.named_parameters())[n] for n in PNAMES]
    preds, alphas = AttentionDecoderFn.apply(dec, enc, caps, decode_lengths, *params)
    return preds, encoded_captions, decode_lengths, alphas


class FusedStepState:
    """Per-shape buffers of the fused loss (loss rows, lse, time-major dlogits, reg)."""

    def __init__(self):
        self.key = None

    def get(self, B, T, V, P, device):
        key = (B, T, V, P, str(device))
        if key != self.key:
            f = dict(device=device, dtype=torch.float32)
            self.loss_rows = torch.empty(B * T, **f)
            self.dlogits = torch.empty(T * B, V, **f)
            self.reg = torch.empty(K.alpha_reg_parts(B, P), **f)
            self.dreg = torch.empty(B, P, **f)
            self.loss = torch.empty(1, **f)
            self.key = key
        return self


_FS = FusedStepState()


def fused_loss_and_grads(dec, encoder_out, captions, caption_lengths, alpha_c, grads, need=None,
                         seed_dev=None, denc=None, on_fc_grads=None):
    """Forward + loss + backward of one decoder training step (models/attention.py:393-420).

    Writes d(loss)/d(param) into ``grads`` (name -> tensor, e.g. the optimizer's flat
    views); returns (loss (1,) device tensor, predictions, alphas). ``seed_dev``: an int64
    device counter driving the dropout mask (graph-replayable); else a host seed is drawn.
    ``denc``: optional (B,14,14,2048)-sized buffer receiving d(loss)/d(encoder_out) (fine-tune).
    ``on_fc_grads``: callback once the fc gradients are final (before the BPTT loop)."""
    enc, caps = _prep_inputs(dec, encoder_out, captions)
    p = decoder_params(dec)
    decode_lengths = [int(l) - 1 for l in caption_lengths]
    drop = dec.dropout.p if dec.training else 0.0
    host_seed = 0x5EED if seed_dev is not None else (_seed() if drop > 0 else 0)
    preds, alphas, st = CORE.forward(p, enc, caps, decode_lengths, dropout_p=drop, training=dec.training,
                                     seed=host_seed, seed_dev=seed_dev, emb_dense=dense_embeddings(dec, caps))
    _GEN[0] += 1
    dm = st["dm"]
    B, T, V, P, L = dm.B, dm.T, dm.V, dm.P, dm.L
    fs = _FS.get(B, T, V, P, enc.device)
    nrows = sum(decode_lengths)
    # CE over the packed rows (no ignore_index: pads are scored, Q2) -> time-major dlogits
    K.ce_fwd_bwd(preds, caps, B, T, L, V, st["bt_dev"], nrows, fs.loss_rows, None, fs.dlogits,
                 dl_time_major=True)
    K.alpha_reg(alphas, B, T, P, alpha_c, fs.reg, fs.dreg)
    K.loss_finalize(fs.loss_rows, B * T, nrows, fs.reg, fs.loss)
    g = {n: grads[n] for n in (need if need is not None else grads)
         if not (st["dense_emb"] and n == "embedding.weight")}
    if "attention.full_att.weight" in g:
        g["attention.full_att.weight"] = g["attention.full_att.weight"].view(-1)
    CORE.backward(p, st, g, fs.dlogits, dpred_time_major=True, dreg=fs.dreg,
                  denc=None if denc is None else denc.view(B, P, -1), on_fc_grads=on_fc_grads)
    return fs.loss, preds, alphas


# ----------------------------------------------------------------------------------------
# inference-only pieces
# ----------------------------------------------------------------------------------------
def _linear(x2d, W, b, out=None):
    M, Kd = x2d.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x2d.device, dtype=torch.float32)
    K.gemm(K.problem(M, N, Kd, x2d, Kd, W, Kd, out, N, bias=b), CAPMI_A_KMAJOR, CAPMI_B_NMAJOR_W,
           K.TILE_128 if M >= 512 else K.TILE_64)
    return out


def _no_grad_check(*params):
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        raise NotImplementedError(
            "capmi: the standalone SoftAttention / init_hidden_state are inference kernels; "
            "training goes through AttentionDecoder.forward (run them under torch.no_grad())")


def soft_attention_forward(att, encoder_out, decoder_hidden):
    """models/attention.py:43-61 for one step: (B,P,E),(B,D) -> awe (B,E), alpha (B,P)."""
    _no_grad_check(*att.parameters())
    enc = encoder_out.contiguous()
    h = decoder_hidden.contiguous()
    B, P, E = enc.shape
    A = att.enc_att.out_features
    att_enc = _linear(enc.view(B * P, E), att.enc_att.weight, att.enc_att.bias)
    att_dec = _linear(h, att.dec_att.weight, att.dec_att.bias)
    e = torch.empty(B, P, device=enc.device, dtype=torch.float32)
    K.att_score_fwd(att_enc, att_dec, 1, 0, None, att.full_att.weight.view(-1), att.full_att.bias, B, P, A, e)
    alpha = torch.empty(B, P, device=enc.device, dtype=torch.float32)
    awe = torch.empty(B, E, device=enc.device, dtype=torch.float32)
    K.att_softmax_ctx_fwd(e, enc, B, P, E, B, alpha, P, awe)
    return awe, alpha


def init_hidden_forward(dec, encoder_out):
    """models/attention.py:151-164: mean over P, then h_lin / c_lin."""
    _no_grad_check(dec.h_lin.weight, dec.c_lin.weight)
    enc = encoder_out.contiguous()
    B, P, E = enc.shape
    mean = torch.empty(B, E, device=enc.device, dtype=torch.float32)
    K.mean_rows(enc, B, P, E, mean)
    return _linear(mean, dec.h_lin.weight, dec.h_lin.bias), _linear(mean, dec.c_lin.weight, dec.c_lin.bias)
