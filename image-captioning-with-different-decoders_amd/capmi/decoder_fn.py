"""Autograd entry points and fused loss for the attention decoder.

* ``AttentionDecoderFn``: the differentiable ``AttentionDecoder.forward`` the
  reference's own training loop calls (models/attention.py:396): returns
  (predictions, alphas); its backward runs the capmi BPTT kernels.
* ``fused_loss_and_grads``: the whole loss of models/attention.py:401-414 (CE
  over the packed rows incl. pads + the doubly-stochastic regulariser) and the
  full decoder backward in one go, writing parameter gradients straight into the
  optimizer's flat buffer -- what capmi's own ``train()`` and bench.py run.
* ``soft_attention_forward`` / ``init_hidden_forward``: the standalone sub-modules
  (beam search uses them, gen_captions.py:62-72), differentiable through
  ``SoftAttentionFn`` / ``InitHiddenFn`` on the decoder's own step kernels.
"""
import torch

from . import kernels as K
from ._lib import CAPMI_A_KMAJOR, CAPMI_A_MMAJOR as AMM, CAPMI_B_KROWS as BKR, CAPMI_B_NMAJOR_W
from ._lib import CAPMI_GEMM_BF16, CAPMI_GEMM_SPLIT3
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


def gemm_flags(dec):
    """Operand staging of the decoder's GEMMs for ``dec.compute_precision`` (models/attention.py
    set_compute_precision): 'fp32' -> fp32 MFMA, 'fp32-x3' -> CAPMI_GEMM_SPLIT3 (fp32-accurate),
    'bf16' -> CAPMI_GEMM_BF16."""
    prec = getattr(dec, "compute_precision", "fp32")
    return {"fp32": 0, "fp32-x3": CAPMI_GEMM_SPLIT3, "bf16": CAPMI_GEMM_BF16}[prec]


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
                                         emb_dense=dense_embeddings(dec, caps), gemm_flags=gemm_flags(dec))
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
            self.dreg_q = torch.empty(B, P, **f)  # the distinct rows' share (dup > 1), <= P
            self.loss = torch.empty(1, **f)
            self.key = key
        return self


_FS = FusedStepState()


def fused_loss_and_grads(dec, encoder_out, captions, caption_lengths, alpha_c, grads, need=None,
                         seed_dev=None, denc=None, on_fc_grads=None, dup=1):
    """Forward + loss + backward of one decoder training step (models/attention.py:393-420).

    Writes d(loss)/d(param) into ``grads`` (name -> tensor, e.g. the optimizer's flat
    views); returns (loss (1,) device tensor, predictions, alphas). ``seed_dev``: an int64
    device counter driving the dropout mask (graph-replayable); else a host seed is drawn.
    ``denc``: optional buffer shaped like ``encoder_out`` receiving d(loss)/d(encoder_out) (fine-tune;
    with ``dup`` the gradient of the F x F map).
    ``on_fc_grads``: callback once the fc gradients are final (before the BPTT loop).
    ``dup`` > 1: ``encoder_out`` is the (B, F, F, E) map whose pooled (B, F dup, F dup, E) form the
    reference would decode (every pooled pixel repeated dup x dup times, DecoderCore.forward); the
    loss, predictions and alphas (B, T, (F dup)^2) are the pooled form's."""
    enc, caps = _prep_inputs(dec, encoder_out, captions)
    p = decoder_params(dec)
    decode_lengths = [int(l) - 1 for l in caption_lengths]
    drop = dec.dropout.p if dec.training else 0.0
    host_seed = 0x5EED if seed_dev is not None else (_seed() if drop > 0 else 0)
    preds, alphas, st = CORE.forward(p, enc, caps, decode_lengths, dropout_p=drop, training=dec.training,
                                     seed=host_seed, seed_dev=seed_dev, emb_dense=dense_embeddings(dec, caps),
                                     dup=dup, gemm_flags=gemm_flags(dec))
    _GEN[0] += 1
    dm = st["dm"]
    B, T, V, L = dm.B, dm.T, dm.V, dm.L
    P = alphas.shape[2]  # the reference's positions ((F dup)^2 with dup)
    fs = _FS.get(B, T, V, P, enc.device)
    nrows = sum(decode_lengths)
    # CE over the packed rows (no ignore_index: pads are scored, Q2) -> time-major dlogits
    K.ce_fwd_bwd(preds, caps, B, T, L, V, st["bt_dev"], nrows, fs.loss_rows, None, fs.dlogits,
                 dl_time_major=True)
    K.alpha_reg(alphas, B, T, P, alpha_c, fs.reg, fs.dreg)
    K.loss_finalize(fs.loss_rows, B * T, nrows, fs.reg, fs.loss)
    dreg = fs.dreg
    if dup > 1:
        # d(loss)/d(alpha_q) of a distinct row: the group's dup^2 equal positions each contribute
        # dreg_p / dup^2 -- the value at one representative
        K.att_dup_pick(fs.dreg, B, st["F"], dup, fs.dreg_q)
        dreg = fs.dreg_q
    g = {n: grads[n] for n in (need if need is not None else grads)
         if not (st["dense_emb"] and n == "embedding.weight")}
    if "attention.full_att.weight" in g:
        g["attention.full_att.weight"] = g["attention.full_att.weight"].view(-1)
    CORE.backward(p, st, g, fs.dlogits, dpred_time_major=True, dreg=dreg,
                  denc=None if denc is None else denc.view(B, dm.P, -1), on_fc_grads=on_fc_grads)
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


def _colsum(x2d, rows, cols, out):
    work = torch.empty(K.colsum_work_size(rows, cols), device=x2d.device, dtype=torch.float32)
    K.colsum(x2d, rows, cols, cols, out, work)
    return out


def _gemm_t(dY, X, rows, n_out, n_in):
    """d(W) = dY^T X for Y = X W^T: dY (rows, n_out), X (rows, n_in) -> (n_out, n_in)."""
    out = torch.empty(n_out, n_in, device=dY.device, dtype=torch.float32)
    K.gemm(K.problem(n_out, n_in, rows, dY, n_out, X, n_in, out, n_in), AMM, BKR, K.TILE_128)
    return out


def _gemm_back(dY, W, rows, n_out, n_in, out=None, beta=0.0):
    """d(X) (+)= dY W for Y = X W^T: dY (rows, n_out), W (n_out, n_in) -> (rows, n_in)."""
    if out is None:
        out = torch.empty(rows, n_in, device=dY.device, dtype=torch.float32)
    K.gemm(K.problem(rows, n_in, n_out, dY, n_out, W, n_in, out, n_in, beta=beta), CAPMI_A_KMAJOR, BKR,
           K.TILE_128 if rows >= 512 else K.TILE_64)
    return out


def _f32_dev(*ts):
    for t in ts:
        if not t.is_cuda or t.dtype != torch.float32:
            raise TypeError("capmi SoftAttention / init_hidden_state take float32 HIP tensors")


class SoftAttentionFn(torch.autograd.Function):
    """models/attention.py:43-61 for one step, differentiable: the forward kernels of the decoder
    step (score, softmax + context) and, for the backward, its BPTT kernels at T = 1
    (att_ctx_bwd, att_score_bwd, att_enc_grad, att_enc_dinput) plus the weight-gradient GEMMs."""

    @staticmethod
    def forward(ctx, enc, h, w_enc, b_enc, w_dec, b_dec, wf, bf):
        B, P, E = enc.shape
        A = w_enc.shape[0]
        att_enc = _linear(enc.view(B * P, E), w_enc, b_enc)
        att_dec = _linear(h, w_dec, b_dec)
        e = torch.empty(B, P, device=enc.device, dtype=torch.float32)
        K.att_score_fwd(att_enc, att_dec, 1, 0, None, wf.reshape(-1), bf, B, P, A, e)
        alpha = torch.empty(B, P, device=enc.device, dtype=torch.float32)
        awe = torch.empty(B, E, device=enc.device, dtype=torch.float32)
        K.att_softmax_ctx_fwd(e, enc, B, P, E, B, alpha, P, awe)
        ctx.save_for_backward(enc, h, w_enc, w_dec, wf, att_enc, att_dec, alpha, awe)
        ctx.wf_shape = wf.shape
        return awe, alpha

    @staticmethod
    def backward(ctx, dawe, dalpha_out):
        enc, h, w_enc, w_dec, wf, att_enc, att_dec, alpha, awe = ctx.saved_tensors
        B, P, E = enc.shape
        A, D = w_enc.shape[0], h.shape[1]
        f = dict(device=enc.device, dtype=torch.float32)
        dawe = torch.zeros(B, E, **f) if dawe is None else dawe.contiguous()
        dalpha = torch.empty(B, P, **f)
        # dalpha[b][p] = dawe . enc[b][p] (no gate here), then softmax + ReLU-score backward
        K.att_ctx_bwd(dawe, 1, 0, None, None, enc, B, P, E, None, dalpha)
        dr = None if dalpha_out is None else dalpha_out.contiguous()
        de = torch.empty(B, P, **f)
        dad = torch.empty(B, A, **f)
        K.att_score_bwd(dalpha, dr, P, alpha, P, att_enc, att_dec, wf.reshape(-1), B, P, A, B, de, dad)
        nblk = K.att_enc_grad_blocks(B, P)
        datt = torch.empty(B * P, A, **f)
        wf_part, bf_part = torch.empty(nblk, A, **f), torch.empty(nblk, 1, **f)
        nblk = K.att_enc_grad(de, att_enc, att_dec, wf.reshape(-1), 1, B, P, A, datt, wf_part, bf_part)
        need = ctx.needs_input_grad
        g_enc = g_h = None
        if need[0]:
            g_enc = torch.empty(B, P, E, **f)
            K.att_enc_dinput(alpha, P, dawe, None, B, 1, P, E, g_enc)  # context sums (:59-60)
            _gemm_back(datt, w_enc, B * P, A, E, out=g_enc.view(B * P, E), beta=1.0)  # enc_att (:54)
        if need[1]:
            g_h = _gemm_back(dad, w_dec, B, A, D)
        g_wenc = _gemm_t(datt, enc.view(B * P, E), B * P, A, E) if need[2] else None
        g_benc = _colsum(datt, B * P, A, torch.empty(A, **f)) if need[3] else None
        g_wdec = _gemm_t(dad, h, B, A, D) if need[4] else None
        g_bdec = _colsum(dad, B, A, torch.empty(A, **f)) if need[5] else None
        g_wf = _colsum(wf_part, nblk, A, torch.empty(A, **f)).view(ctx.wf_shape) if need[6] else None
        g_bf = _colsum(bf_part, nblk, 1, torch.empty(1, **f)) if need[7] else None
        return g_enc, g_h, g_wenc, g_benc, g_wdec, g_bdec, g_wf, g_bf


def soft_attention_forward(att, encoder_out, decoder_hidden):
    """models/attention.py:43-61 for one step: (B,P,E),(B,D) -> awe (B,E), alpha (B,P);
    differentiable in every input and parameter (SoftAttentionFn)."""
    enc = encoder_out.contiguous()
    h = decoder_hidden.contiguous()
    _f32_dev(enc, h)
    return SoftAttentionFn.apply(enc, h, att.enc_att.weight, att.enc_att.bias, att.dec_att.weight,
                                 att.dec_att.bias, att.full_att.weight, att.full_att.bias)


class InitHiddenFn(torch.autograd.Function):
    """models/attention.py:151-164: mean over P, then h_lin / c_lin; differentiable."""

    @staticmethod
    def forward(ctx, enc, w_h, b_h, w_c, b_c):
        B, P, E = enc.shape
        mean = torch.empty(B, E, device=enc.device, dtype=torch.float32)
        K.mean_rows(enc, B, P, E, mean)
        ctx.save_for_backward(mean, w_h, w_c)
        ctx.P = P
        return _linear(mean, w_h, b_h), _linear(mean, w_c, b_c)

    @staticmethod
    def backward(ctx, dh0, dc0):
        mean, w_h, w_c = ctx.saved_tensors
        B, E = mean.shape
        D, P = w_h.shape[0], ctx.P
        f = dict(device=mean.device, dtype=torch.float32)
        dh0 = torch.zeros(B, D, **f) if dh0 is None else dh0.contiguous()
        dc0 = torch.zeros(B, D, **f) if dc0 is None else dc0.contiguous()
        need = ctx.needs_input_grad
        g_enc = None
        if need[0]:
            dmean = _gemm_back(dh0, w_h, B, D, E)
            _gemm_back(dc0, w_c, B, D, E, out=dmean, beta=1.0)
            g_enc = torch.empty(B, P, E, **f)
            # denc = dmean / P on every pixel (the context term of the kernel is fed zeros)
            K.att_enc_dinput(torch.zeros(B, P, **f), P, torch.zeros(B, E, **f), dmean, B, 1, P, E, g_enc)
        g_wh = _gemm_t(dh0, mean, B, D, E) if need[1] else None
        g_bh = _colsum(dh0, B, D, torch.empty(D, **f)) if need[2] else None
        g_wc = _gemm_t(dc0, mean, B, D, E) if need[3] else None
        g_bc = _colsum(dc0, B, D, torch.empty(D, **f)) if need[4] else None
        return g_enc, g_wh, g_bh, g_wc, g_bc


def init_hidden_forward(dec, encoder_out):
    """models/attention.py:151-164: mean over P, then h_lin / c_lin (differentiable)."""
    enc = encoder_out.contiguous()
    _f32_dev(enc)
    return InitHiddenFn.apply(enc, dec.h_lin.weight, dec.h_lin.bias, dec.c_lin.weight, dec.c_lin.bias)
