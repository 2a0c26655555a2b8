"""The baseline decoder (reference models/baseline.py:24-111) on the capmi kernels: an LSTM over
[image feature, embedding(captions[:, :-1])] with teacher forcing, then Linear to the vocabulary.

SURVEY.md §8f rank 4. The step is the attention decoder's minus the attention: the input half of
the LSTM GEMM is hoisted over all T steps (one (T*B) x 4H x M GEMM, both LSTM biases in its
epilogue), each step adds h_{t-1} W_hh^T and runs the fused cell (capmi_lstm_cell_fwd, gate order
i,f,g,o as torch.nn.LSTM), and the vocabulary projection is one (T*B) x V x H GEMM written
batch-first (row remap) after the loop. The backward is BPTT with the same kernels the attention
decoder uses (capmi_lstm_cell_bwd, the recurrent dh GEMM per step, hoisted weight gradients,
embedding scatter-add). State is time-major: X[t][b][M], H[t][b][H], C, ACT[t][b][4H].
"""
import torch

from . import kernels as K
from ._lib import CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_B_KROWS, CAPMI_B_NMAJOR_W

AK, AMM, BW, BKR = CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_B_NMAJOR_W, CAPMI_B_KROWS


def _params(dec):
    lstm = dec.lstm
    return (dec.embedding.weight, lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0,
            dec.linear.weight, dec.linear.bias)


class BaselineDecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dec, img_features, captions, *params):
        emb_w, w_ih, w_hh, b_ih, b_hh, w_lin, b_lin = params
        B, L = captions.shape
        T, M, Hd, V = L, dec.embed_size, dec.hidden_size, w_lin.shape[0]
        dev = img_features.device
        f = dict(device=dev, dtype=torch.float32)
        caps = captions.contiguous()
        X = torch.empty(T, B, M, **f)
        X[0].copy_(img_features.float())  # step 0 = the image feature (reference :104)
        if T > 1:  # steps 1.. = embedding(captions[:, :-1]) (reference :98-101)
            K.embed_gather(emb_w, caps, B, L, T - 1, X[1:], M)
        GX = torch.empty(T * B, 4 * Hd, **f)
        K.gemm_sk(K.problem(T * B, 4 * Hd, M, X, M, w_ih, M, GX, 4 * Hd, bias=b_ih, bias2=b_hh), AK,
                  dec._capmi_ws(dev), K.TILE_AUTO)
        H = torch.empty(T, B, Hd, **f)
        C = torch.empty(T, B, Hd, **f)
        ACT = torch.empty(T, B, 4 * Hd, **f)
        HH = torch.empty(B, 4 * Hd, **f)
        zeros = torch.zeros(B, Hd, **f)
        for t in range(T):
            if t > 0:
                K.gemm(K.problem(B, 4 * Hd, Hd, H[t - 1], Hd, w_hh, Hd, HH, 4 * Hd), AK, BW, K.TILE_64)
            K.lstm_cell_fwd(GX[t * B:], 1, 0, None, HH if t > 0 else None, 1 if t > 0 else 0, 0,
                            C[t - 1] if t > 0 else zeros, B, Hd, H[t], C[t], ACT[t])
        out = torch.empty(B, T, V, **f)
        # row r = t*B + b of the (T*B, V) product lands at out[b][t]: remap (r % B)*T*V + (r / B)*V
        K.gemm_sk(K.problem(T * B, V, Hd, H, Hd, w_lin, Hd, out, T * V, c_r1=B, c_s2=V, bias=b_lin), AK,
                  dec._capmi_ws(dev), K.TILE_AUTO)
        ctx.dec = dec
        ctx.dims = (B, L, T, M, Hd, V)
        ctx.img_dtype = img_features.dtype
        ctx.save_for_backward(caps, X, H, C, ACT, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        caps, X, H, C, ACT, emb_w, w_ih, w_hh, b_ih, b_hh, w_lin, b_lin = ctx.saved_tensors
        B, L, T, M, Hd, V = ctx.dims
        dev = X.device
        f = dict(device=dev, dtype=torch.float32)
        ws = ctx.dec._capmi_ws(dev)
        dout = dout.float().contiguous()  # (B, T, V)
        # dH[t*B+b] = dout[b][t] . W_lin   (A rows remapped from batch-first)
        dH = torch.empty(T * B, Hd, **f)
        K.gemm_sk(K.problem(T * B, Hd, V, dout, T * V, w_lin, Hd, dH, Hd, a_r1=B, a_s2=V), AK, ws, K.TILE_AUTO,
                  bmode=BKR)
        g_lin = torch.empty_like(w_lin) if w_lin.requires_grad else None
        if g_lin is not None:  # dW_lin = dout^T H over the (T*B) rows
            K.gemm_sk(K.problem(V, Hd, T * B, dout, T * V, H, Hd, g_lin, Hd, a_r1=B, a_s2=V), AMM, ws, K.TILE_AUTO,
                      bmode=BKR)
        g_blin = None
        if b_lin.requires_grad:
            g_blin = torch.empty_like(b_lin)
            K.colsum(dout, B * T, V, V, g_blin, torch.empty(K.colsum_work_size(B * T, V), **f))
        # BPTT
        DG = torch.empty(T, B, 4 * Hd, **f)
        DHR = torch.empty(B, Hd, **f)
        DC = [torch.empty(B, Hd, **f), torch.empty(B, Hd, **f)]
        zeros = torch.zeros(B, Hd, **f)
        for t in range(T - 1, -1, -1):
            dc_in = DC[(t + 1) & 1] if t < T - 1 else None
            K.lstm_cell_bwd(dH[t * B:], DHR, 1 if t < T - 1 else 0, 0, dc_in, ACT[t], C[t - 1] if t > 0 else zeros,
                            C[t], B, Hd, B, DG[t], DC[t & 1])
            if t > 0:  # dh_{t-1} (recurrent part) = dgates_t . W_hh
                K.gemm(K.problem(B, Hd, 4 * Hd, DG[t], 4 * Hd, w_hh, Hd, DHR, Hd), AK, BKR, K.TILE_64)
        g_ih = g_hh = g_bih = g_bhh = None
        if w_ih.requires_grad:
            g_ih = torch.empty_like(w_ih)  # dW_ih = DG^T X
            K.gemm_sk(K.problem(4 * Hd, M, T * B, DG, 4 * Hd, X, M, g_ih, M), AMM, ws, K.TILE_AUTO, bmode=BKR)
        if w_hh.requires_grad:
            g_hh = torch.zeros_like(w_hh) if T == 1 else torch.empty_like(w_hh)
            if T > 1:  # dW_hh = sum_{t>=1} DG[t]^T H[t-1]
                K.gemm_sk(K.problem(4 * Hd, Hd, (T - 1) * B, DG[1:], 4 * Hd, H, Hd, g_hh, Hd), AMM, ws, K.TILE_AUTO,
                          bmode=BKR)
        if b_ih.requires_grad or b_hh.requires_grad:
            gb = torch.empty(4 * Hd, **f)
            K.colsum(DG, T * B, 4 * Hd, 4 * Hd, gb, torch.empty(K.colsum_work_size(T * B, 4 * Hd), **f))
            g_bih = gb if b_ih.requires_grad else None
            g_bhh = gb.clone() if b_hh.requires_grad else None
        # dX = DG . W_ih: step 0 -> the image feature, steps 1.. -> the embedding rows
        DX = torch.empty(T, B, M, **f)
        K.gemm_sk(K.problem(T * B, M, 4 * Hd, DG, 4 * Hd, w_ih, M, DX, M), AK, ws, K.TILE_AUTO, bmode=BKR)
        g_img = DX[0].to(ctx.img_dtype) if ctx.needs_input_grad[1] else None
        g_emb = None
        if emb_w.requires_grad and T > 1:
            g_emb = torch.zeros_like(emb_w)
            K.embed_scatter_add(DX[1:], M, caps, B, L, T - 1, None, M, g_emb)
        return (None, g_img, None, g_emb, g_ih, g_hh, g_bih, g_bhh, g_lin, g_blin)


def baseline_forward(dec, img_features, captions):
    if not (img_features.is_cuda and captions.is_cuda):
        raise RuntimeError("capmi baseline decoder path needs HIP tensors")
    if captions.dtype != torch.int64:
        raise TypeError("captions must be int64")
    return BaselineDecoderFn.apply(dec, img_features.contiguous(), captions, *_params(dec))
