"""Forward and backward-through-time of the soft-attention LSTM decoder on libcapmi.

Restates models/attention.py:218-284 (AttentionDecoder.forward) and, for the
backward pass, what autograd does through it, with the loop-invariant work
hoisted out of the 24-step recurrence:

  * ``enc_att(encoder_out)`` (:54, recomputed every step by the reference, Q5)
    is one GEMM before the loop; its weight gradient is one GEMM after it,
    over d(att_enc) summed over t (exact in math, different fp32 sum order);
  * the embedding half of ``W_ih`` (teacher forcing) is one GEMM for all t;
  * ``fc`` (:279) is one (T*B) x D x V GEMM after the loop, dW_fc one GEMM;
  * every weight gradient of the recurrent GEMMs is one GEMM over the stacked
    per-step gradients after the loop.

Per timestep there remain 5 launches forward (grouped h-GEMM, score, softmax +
context + gate, x-GEMM, LSTM pointwise) and 5 backward. Per-step state is
time-major ([t][b][...]); the returned predictions/alphas keep the reference's
batch-major (B,T,V)/(B,T,P) layouts.

Ragged captions follow the reference's ``batch_size_t = sum(l > t)`` rule
(:261): rows b >= bt[t] produce zero predictions/alphas and no gradient.
"""
import math
import os

import torch

from . import kernels as K
from ._lib import CAPMI_A_KMAJOR as AK, CAPMI_A_MMAJOR as AMM, CAPMI_B_KROWS as BKR
from ._lib import CAPMI_B_NMAJOR_W as BW, CAPMI_GEMM_BF16, CAPMI_GEMM_SPLIT3
from ._lib import CAPMI_DSTEP_GATE_BWD, CAPMI_DSTEP_LSTM_BWD, CAPMI_DSTEP_LSTM_FWD, CAPMI_DSTEP_STORE2

E_DIM = 2048
PNAMES = ["attention.enc_att.weight", "attention.enc_att.bias", "attention.dec_att.weight",
          "attention.dec_att.bias", "attention.full_att.weight", "attention.full_att.bias",
          "decode_step.weight_ih", "decode_step.weight_hh", "decode_step.bias_ih",
          "decode_step.bias_hh", "h_lin.weight", "h_lin.bias", "c_lin.weight", "c_lin.bias",
          "f_beta.weight", "f_beta.bias", "fc.weight", "fc.bias", "embedding.weight"]


def _dsplit(M, N, nt, K_, target=None):
    """k-split of a capmi_dstep_gemm launch: tiles * S ~ target workgroups, each workgroup at most
    16 k-tiles (4 k-groups x 4 loaded up front; the C side raises S to that too), >= 1 per split."""
    target = target or int(os.environ.get("CAPMI_DSTEP_WGS", "256"))
    tiles = -(-M // 64) * (N // nt)
    kt = K_ // 32
    return max(1, min(kt, max(-(-kt // 16), round(target / tiles))))


# round 6: the hoisted weight gradients dW = dY^T X (rows = timesteps x batch) on gemm_x3w, the encoder fine-tune's
# weight-gradient kernel (both fp32 operands split in-kernel, 256 x 128 tiles, k-split slabs) -- in the x3
# arithmetic, or with one bf16 term per operand in the bf16 configuration (gemm_w16) -- where its planner takes the
# problem (CAPMI_DEC_WGRAD_X3W=0: the split-staging stream-K kernel, A/B)
DEC_WGRAD_X3W = os.environ.get("CAPMI_DEC_WGRAD_X3W", "1") != "0"

# workgroups a per-timestep GEMM launch aims for (CAPMI_DEC_WGS, A/B measurement: fewer, longer
# workgroups leave more CUs to the encoder stream running beside the decoder)
DEC_WGS = int(os.environ.get("CAPMI_DEC_WGS", "256"))


def _split(M, N, K_, tile, target=None, min_k=128):
    """K-split so that tiles*split ~ target workgroups (each split keeps >= min_k of K)."""
    target = DEC_WGS if target is None else target
    t = K.tiles_for(M, N, tile)
    if t >= target:
        return 1
    s = max(1, min(math.ceil(target / t), K_ // min_k))
    return s


class DecoderDims:
    def __init__(self, B, T, L, P, A, D, M, V, E=E_DIM, gemm_flags=0):
        self.B, self.T, self.L, self.P, self.A, self.D, self.M, self.V, self.E = B, T, L, P, A, D, M, V, E
        self.X = M + E
        for name, v in (("A", A), ("D", D), ("M", M), ("E", E)):
            if v % 4:
                raise ValueError(f"capmi decoder needs {name} % 4 == 0 (got {v})")
        if A > 1024:
            raise ValueError("capmi decoder supports attention_dim <= 1024")
        # split-K factors of the per-step (M = B) GEMMs
        self.s_h = (_split(B, A, D, K.TILE_64), _split(B, E, D, K.TILE_64), _split(B, 4 * D, D, K.TILE_64))
        self.s_x = _split(B, 4 * D, E, K.TILE_64)
        self.s_dx = _split(B, E, 4 * D, K.TILE_64)
        self.s_dh = (_split(B, D, 4 * D, K.TILE_64, DEC_WGS * 3 // 8), _split(B, D, E, K.TILE_64, DEC_WGS * 3 // 8),
                     _split(B, D, A, K.TILE_64, DEC_WGS // 4))
        # decoder_step.hip (CAPMI_DEC_FUSED): "1" (default since round 6) the attention forward (score +
        # softmax + context + gate) and backward (gate split + context + softmax + score) as one launch
        # each, reading the split-K GEMM partials; "2" also the last-arriver GEMMs with the LSTM cell in
        # their epilogue (three launches per timestep each way); "0" the five-launch path. Measured
        # (DESIGN.md 4.5): through round 5 "1" was 0.9 % faster alone but 1.1 % slower in the pipelined
        # step; with the encoder stream at high priority (round 6) it is ahead in the pipelined step
        # too on every interleaved round (config 2 6214 -> 6245, config 4 2151 -> 2157 img/s, same box), but
        # not with the bf16 GEMMs (config 5 13096 -> 12767): default "1" except for CAPMI_GEMM_BF16; "2" stays
        # 5 % slower
        mode = os.environ.get("CAPMI_DEC_FUSED", "0" if gemm_flags == CAPMI_GEMM_BF16 else "1")
        self.fused_att = mode != "0" and P <= 56 and E + P + 4100 <= 16384
        self.fused = (mode == "2" and self.fused_att and A % 32 == 0 and D % 32 == 0 and E % 64 == 0
                      and M % 4 == 0)
        if self.fused:
            self.f_s1 = _dsplit(B, A + E, 32, D)              # att_dec | f_beta from h
            self.f_s3 = _dsplit(B, 4 * D, 64, E + D)          # [gate*awe | h] x [W_ih_awe | W_hh] + LSTM
            self.f_sb1 = _dsplit(B, D, 16, 4 * D + E + A)     # dh of step t+1 + LSTM backward of step t
            self.f_sb2 = _dsplit(B, E, 64, 4 * D)             # d(gate*awe) + gate / context split
            self.f_part = max(-(-B // 64) * n * s * 64 * nt for n, s, nt in (
                ((A + E) // 32, self.f_s1, 32), (D // 16, self.f_s3, 64), (D // 16, self.f_sb1, 16),
                (E // 64, self.f_sb2, 64)))

    def key(self):
        return (self.B, self.T, self.L, self.P, self.A, self.D, self.M, self.V, self.E)


class Workspace:
    """All decoder buffers for one shape, allocated once (graph-capture friendly)."""

    def __init__(self, dm, device):
        B, T, P, A, D, M, V, E, X = dm.B, dm.T, dm.P, dm.A, dm.D, dm.M, dm.V, dm.E, dm.X
        f = dict(device=device, dtype=torch.float32)
        e = torch.empty
        self.X = e(T, B, X, **f)
        self.mean = e(B, E, **f)
        self.H = e(T + 1, B, D, **f)
        self.C = e(T + 1, B, D, **f)
        self.ACT = e(T, B, 4 * D, **f)
        self.AD = e(T, B, A, **f)
        self.AWE = e(T, B, E, **f)
        self.GATE = e(T, B, E, **f)
        self.XEMB = e(T, B, 4 * D, **f)
        self.ATT_ENC = e(B, P, A, **f)
        self.score = e(B, P, **f)
        s_a, s_g, s_hh = dm.s_h
        self.P_ad = e(s_a, B, A, **f)
        self.P_gate = e(s_g, B, E, **f)
        self.P_hh = e(s_hh, B, 4 * D, **f)
        self.P_x = e(dm.s_x, B, 4 * D, **f)
        # backward
        self.DHD = e(T, B, D, **f)
        self.DG = e(T, B, 4 * D, **f)
        self.DGP = e(T, B, E, **f)
        self.DAD = e(T, B, A, **f)
        self.DE = e(T, B, P, **f)
        self.DALPHA = e(B, P, **f)
        self.DC = e(2, B, D, **f)
        self.P_dx = e(dm.s_dx, B, E, **f)
        self.P_dh = e(sum(dm.s_dh), B, D, **f)
        self.DH0 = e(B, D, **f)
        self.DATT = e(B, P, A, **f)
        nblk = K.att_enc_grad_blocks(B, P)
        self.WF_PART = e(nblk, A, **f)
        self.BF_PART = e(nblk, 1, **f)
        # generic scratch: split-K slabs of the hoisted GEMMs and colsum work
        self.scratch = e(max(8 * T * B * D, 32 * B * D, T * B * M, 256 * 128 * 128), **f)
        self.sk = K.gemm_workspace(device)  # stream-K workspace of the hoisted GEMMs
        self.work = e(max(K.colsum_work_size(T * B, V), K.colsum_work_size(B * P, A),
                          K.colsum_work_size(T * B, 4 * D), K.colsum_work_size(T * B, E), 64), **f)
        if dm.fused:
            self.f_part = e(dm.f_part, **f)
            # last-arriver counters of the GEMM tiles; every launch leaves them zero
            self.f_count = torch.zeros(4096, device=device, dtype=torch.int32)
            self.DAWE1 = e(B, E, **f)


class DecoderCore:
    """Stateless apart from the per-shape workspace cache."""

    def __init__(self):
        self._ws = {}

    def workspace(self, dm, device):
        key = (dm.key(), str(device))
        ws = self._ws.get(key)
        if ws is None:
            self._ws.clear()  # one live shape at a time keeps HBM use bounded
            ws = Workspace(dm, device)
            self._ws[key] = ws
        return ws

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _gemm_into(ws, out, ld_out, M, N, Kd, A, lda, B, ldb, amode, bmode, bias=None, gf=0, **kw):
        """C = op(A) op(B) (+bias) for the hoisted (all-timestep) GEMMs: stream-K, so a grid of
        few output tiles (dW_enc_att: 128 tiles of 128x64 over K = B*P) still fills the chip.
        gf: operand staging flags (0 fp32 MFMA, CAPMI_GEMM_SPLIT3, CAPMI_GEMM_BF16)."""
        prob = K.problem(M, N, Kd, A, lda, B, ldb, out, ld_out, bias=bias, **kw)
        if DEC_WGRAD_X3W and amode == AMM and gf in (CAPMI_GEMM_SPLIT3, CAPMI_GEMM_BF16):
            bf16 = gf == CAPMI_GEMM_BF16  # (the bf16 configuration: gemm_w16, one bf16 term per operand)
            if K.gemm_x3w_ok(prob, bmode, bf16):
                K.gemm_x3w(prob, bmode, ws.sk, bf16)
                return
        K.gemm_sk(prob, amode, ws.sk, K.TILE_AUTO, bmode, flags=gf)

    # ------------------------------------------------------------------ fused recurrence
    @staticmethod
    def _fwd_loop_fused(p, dm, ws, enc, bt, alphas):
        """The 24-step loop in three launches per step (decoder_step.hip):
        1. [att_dec | f_beta pre-activation] = h [W_da ; W_fb]^T, last arriver: + bias -> AD[t], sigmoid -> GATE[t]
        2. score + softmax + context + gate * awe -> alphas[:, t], AWE[t], X[t, :, M:]
        3. [gate*awe | h] [W_ih_awe | W_hh]^T (gate-interleaved tiles), last arriver: + xemb, LSTMCell
           -> H[t+1], C[t+1], ACT[t]   (models/attention.py:265-278)"""
        B, T, P, A, D, M, E, X = dm.B, dm.T, dm.P, dm.A, dm.D, dm.M, dm.E, dm.X
        W_ih = p["decode_step.weight_ih"]
        wk1 = torch.cat([p["attention.dec_att.weight"], p["f_beta.weight"]], 0)  # (A + E, D)
        part, cnt = ws.f_part, ws.f_count
        for t in range(T):
            h = ws.H[t]
            K.dstep_gemm([(h, D, wk1, D, D)], B, A + E, 32, dm.f_s1,
                         dict(mode=CAPMI_DSTEP_STORE2, out0=ws.AD[t], ld0=A, bias0=p["attention.dec_att.bias"],
                              nsplit=A, out1=ws.GATE[t], ld1=E, bias1=p["f_beta.bias"], act1=1), part, cnt)
            K.att_fwd_fused(ws.ATT_ENC, ws.AD[t], 0, 0, None, None, p["attention.full_att.weight"],
                            p["attention.full_att.bias"], enc, ws.GATE[t], 0, 0, None, None, B, P, A, E, bt[t],
                            alphas[:, t], T * P, ws.AWE[t], ws.X[t, :, M:], X)
            K.dstep_gemm([(ws.X[t, :, M:], X, W_ih[:, M:], X, E), (h, D, p["decode_step.weight_hh"], D, D)],
                         B, 4 * D, 64, dm.f_s3,
                         dict(mode=CAPMI_DSTEP_LSTM_FWD, D=D, xemb=ws.XEMB[t], c_prev=ws.C[t], h_out=ws.H[t + 1],
                              c_out=ws.C[t + 1], act_out=ws.ACT[t]), part, cnt, gate_D=D)

    @staticmethod
    def _bwd_loop_fused(p, st, dm, ws, enc, bt, dalphas, dreg, denc):
        """Backward through time in three launches per step (decoder_step.hip):
        1. dh_t = DHD[t] + [DG | DGP | DAD]_{t+1} [W_hh ; W_fb ; W_da] (transposed once per call),
           last arriver: LSTMCell backward of step t -> DG[t], dc
        2. d(gate*awe)_t = DG[t] W_ih_awe, last arriver: dawe = d * gate, DGP[t] = d * awe * gate'
        3. dalpha = dawe . enc, last workgroup of each row: softmax + ReLU-score backward -> DE[t], DAD[t]
        The final launch writes dh_0 (h_lin / c_lin backward). Returns the DC slot holding dc_0."""
        B, T, P, A, D, M, E, X = dm.B, dm.T, dm.P, dm.A, dm.D, dm.M, dm.E, dm.X
        W_ih = p["decode_step.weight_ih"]
        wb1 = torch.cat([p["decode_step.weight_hh"].t(), p["f_beta.weight"].t(),
                         p["attention.dec_att.weight"].t()], 1)       # (D, 4D + E + A)
        wb2 = W_ih[:, M:].t().contiguous()                            # (E, 4D)
        KB1 = 4 * D + E + A
        part, cnt = ws.f_part, ws.f_count
        wf = p["attention.full_att.weight"]

        def dh_segs(t1):
            return [(ws.DG[t1], 4 * D, wb1, KB1, 4 * D), (ws.DGP[t1], E, wb1[:, 4 * D:], KB1, E),
                    (ws.DAD[t1], A, wb1[:, 4 * D + E:], KB1, A)]

        cur = 0
        for t in range(T - 1, -1, -1):
            if t == T - 1:
                K.lstm_cell_bwd(ws.DHD[t], None, 0, B * D, None, ws.ACT[t], ws.C[t], ws.C[t + 1], B, D, bt[t],
                                ws.DG[t], ws.DC[cur ^ 1])
            else:
                K.dstep_gemm(dh_segs(t + 1), B, D, 16, dm.f_sb1,
                             dict(mode=CAPMI_DSTEP_LSTM_BWD, D=D, dhd=ws.DHD[t], dc_in=ws.DC[cur], act=ws.ACT[t],
                                  c_prev=ws.C[t], c_cur=ws.C[t + 1], dgates=ws.DG[t], dc_out=ws.DC[cur ^ 1],
                                  bt=bt[t]), part, cnt)
            cur ^= 1
            dawe = ws.DAWE[t] if denc is not None else ws.DAWE1
            K.dstep_gemm([(ws.DG[t], 4 * D, wb2, 4 * D, 4 * D)], B, E, 64, dm.f_sb2,
                         dict(mode=CAPMI_DSTEP_GATE_BWD, gate=ws.GATE[t], awe=ws.AWE[t], dawe_out=dawe,
                              dgp=ws.DGP[t]), part, cnt)
            if dalphas is not None:
                dr, dr_ld = dalphas[:, t], T * P
            elif dreg is not None:
                dr, dr_ld = dreg, P
            else:
                dr, dr_ld = None, 0
            K.att_bwd_fused(dawe, 0, 0, None, None, None, None, enc, st["alphas"][:, t], T * P, dr, dr_ld, ws.ATT_ENC,
                            ws.AD[t], wf, B, P, A, E, bt[t], ws.DE[t], ws.DAD[t])
        K.dstep_gemm(dh_segs(0), B, D, 16, dm.f_sb1, dict(mode=CAPMI_DSTEP_STORE2, out0=ws.DH0, ld0=D, nsplit=D),
                     part, cnt)
        return cur

    # ------------------------------------------------------------------ forward
    def forward(self, p, enc, caps, decode_lengths, *, dropout_p=0.0, training=False, seed=0,
                seed_dev=None, emb_dense=None, dup=1, gemm_flags=0):
        """p: dict name->tensor (PNAMES). enc: (B,P,E) contiguous fp32. caps: (B,L) int64.
        emb_dense: optional (B, Le, M) fp32 word embeddings used instead of the embedding table
        (the BERT variant, :242-244; frozen: no gradient flows into it).
        dup > 1: enc holds the F*F DISTINCT rows of pixel-duplicated features (the reference's
        AdaptiveAvgPool2d of an F x F map to (F dup)^2 positions, models/encoder.py:92,108, repeats
        every pixel dup x dup times). Everything runs on the distinct rows -- the softmax over the
        (F dup)^2 positions is the softmax over the distinct ones / dup^2, the context sum and the
        init mean are unchanged -- and only the returned alphas are expanded.
        gemm_flags: operand staging of every non-fused GEMM, forward and backward: 0 (fp32 MFMA),
        CAPMI_GEMM_SPLIT3 (fp32-accurate three-term split on the bf16 matrix cores) or CAPMI_GEMM_BF16
        (bf16 operands, fp32 accumulation: the bf16 config).
        Returns (predictions (B,T,V), alphas (B,T,P) [P = (F dup)^2 with dup], state)."""
        gf = gemm_flags
        B, P, E = enc.shape
        F = 0
        if dup > 1:
            F = int(round(P ** 0.5))
            if F * F != P:
                raise ValueError(f"dup={dup} needs a square map of distinct rows (got {P})")
        L = caps.shape[1]
        T = max(decode_lengths)
        A = p["attention.enc_att.weight"].shape[0]
        D = p["decode_step.weight_hh"].shape[1]
        M = p["embedding.weight"].shape[1] if emb_dense is None else emb_dense.shape[2]
        V = p["fc.weight"].shape[0]
        dm = DecoderDims(B, T, L, P, A, D, M, V, E, gemm_flags=gf)
        ws = self.workspace(dm, enc.device)
        X = dm.X
        bt = [sum(1 for l in decode_lengths if l > t) for t in range(T)]
        ragged = any(b != B for b in bt)
        bt_dev = torch.tensor(bt, dtype=torch.int32).to(enc.device, non_blocking=True) if ragged else None

        W_ih = p["decode_step.weight_ih"]
        # embeddings of the caption tokens -> X[:, :, :M]      (:247, :273)
        if emb_dense is None:
            K.embed_gather(p["embedding.weight"], caps, B, L, T, ws.X, X)
        else:
            if emb_dense.shape[0] != B or emb_dense.shape[1] < T:
                raise ValueError(f"dense embeddings {tuple(emb_dense.shape)} do not cover (B={B}, T={T})")
            K.embed_dense(emb_dense, T, ws.X, X)
        # init_hidden_state (:151-164)
        K.mean_rows(enc, B, P, E, ws.mean)
        sh = min(8, max(1, E // 256))
        slab = ws.scratch[:2 * sh * B * D]
        K.gemm([K.problem(B, D, E, ws.mean, E, p["h_lin.weight"], E, slab, D, ksplit=sh, c_split_stride=B * D),
                K.problem(B, D, E, ws.mean, E, p["c_lin.weight"], E, slab[sh * B * D:], D, ksplit=sh,
                          c_split_stride=B * D)], AK, BW, K.TILE_64, flags=gf)
        K.splitk_reduce(slab, sh, B * D, B, D, D, ws.H[0], D, bias=p["h_lin.bias"])
        K.splitk_reduce(slab[sh * B * D:], sh, B * D, B, D, D, ws.C[0], D, bias=p["c_lin.bias"])
        # hoisted enc_att (:54) and the embedding half of the LSTM input GEMM
        self._gemm_into(ws, ws.ATT_ENC, A, B * P, A, E, enc, E, p["attention.enc_att.weight"], E, AK, BW,
                        bias=p["attention.enc_att.bias"], gf=gf)
        self._gemm_into(ws, ws.XEMB, 4 * D, T * B, 4 * D, M, ws.X, X, W_ih, X, AK, BW,
                        bias=p["decode_step.bias_ih"], bias2=p["decode_step.bias_hh"], gf=gf)

        alphas = torch.empty(B, T, P, device=enc.device, dtype=torch.float32)  # over the rows enc holds
        s_a, s_g, s_hh = dm.s_h
        W_ih_awe = W_ih[:, M:]
        wf = p["attention.full_att.weight"]
        if dm.fused:
            self._fwd_loop_fused(p, dm, ws, enc, bt, alphas)
        for t in range(T if not dm.fused else 0):
            h = ws.H[t]
            # att_dec (:55), f_beta (:270) and W_hh h (:277) share the input h: one grouped launch
            K.gemm([K.problem(B, A, D, h, D, p["attention.dec_att.weight"], D, ws.P_ad, A, ksplit=s_a,
                              c_split_stride=B * A),
                    K.problem(B, E, D, h, D, p["f_beta.weight"], D, ws.P_gate, E, ksplit=s_g,
                              c_split_stride=B * E),
                    K.problem(B, 4 * D, D, h, D, p["decode_step.weight_hh"], D, ws.P_hh, 4 * D, ksplit=s_hh,
                              c_split_stride=B * 4 * D)], AK, BW, K.TILE_64, flags=gf)
            if dm.fused_att:
                K.att_fwd_fused(ws.ATT_ENC, ws.P_ad, s_a, B * A, p["attention.dec_att.bias"], ws.AD[t], wf,
                                p["attention.full_att.bias"], enc, ws.P_gate, s_g, B * E, p["f_beta.bias"],
                                ws.GATE[t], B, P, A, E, bt[t], alphas[:, t], T * P, ws.AWE[t], ws.X[t, :, M:], X)
            else:
                K.att_score_fwd(ws.ATT_ENC, ws.P_ad, s_a, B * A, p["attention.dec_att.bias"], wf,
                                p["attention.full_att.bias"], B, P, A, ws.score, ws.AD[t])
                K.att_softmax_ctx_fwd(ws.score, enc, B, P, E, bt[t], alphas[:, t], T * P, ws.AWE[t],
                                      ws.P_gate, s_g, B * E, p["f_beta.bias"], ws.GATE[t], ws.X[t, :, M:], X)
            K.gemm(K.problem(B, 4 * D, E, ws.X[t, :, M:], X, W_ih_awe, X, ws.P_x, 4 * D, ksplit=dm.s_x,
                             c_split_stride=B * 4 * D), AK, BW, K.TILE_64, flags=gf)
            K.lstm_cell_fwd(ws.P_x, dm.s_x, B * 4 * D, ws.XEMB[t], ws.P_hh, s_hh, B * 4 * D, ws.C[t], B, D,
                            ws.H[t + 1], ws.C[t + 1], ws.ACT[t])

        # dropout (:107,279) then the hoisted fc over all (t, b) rows
        Hcur = ws.H[1:]
        if training and dropout_p > 0:
            Hd = torch.empty_like(Hcur)
            K.dropout(Hcur, Hcur.numel(), dropout_p, seed, Hd, seed_dev=seed_dev)
        else:
            Hd = Hcur
        preds = torch.empty(B, T, V, device=enc.device, dtype=torch.float32)
        self._gemm_into(ws, preds, T * V, T * B, V, D, Hd, D, p["fc.weight"], D, AK, BW, bias=p["fc.bias"],
                        c_r1=B, c_s2=V, gf=gf)
        if ragged:
            K.mask_rows_tb(preds, bt_dev, T, B, V, T * V, B, V)
        alphas_out = alphas
        if dup > 1:
            alphas_out = torch.empty(B, T, P * dup * dup, device=enc.device, dtype=torch.float32)
            K.att_alpha_expand(alphas, B * T, F, dup, alphas_out)
        state = dict(dm=dm, ws=ws, enc=enc, caps=caps, bt=bt, bt_dev=bt_dev, ragged=ragged, alphas=alphas,
                     dense_emb=emb_dense is not None, dup=dup, F=F, gflags=gf,
                     Hd=Hd, dropout_p=dropout_p if training else 0.0, seed=seed, seed_dev=seed_dev)
        return preds, alphas_out, state

    # ------------------------------------------------------------------ backward
    def backward(self, p, st, grads, dpred, dpred_time_major=False, dreg=None, dalphas=None,
                 need=None, denc=None, on_fc_grads=None):
        """Writes parameter gradients into ``grads`` (dict name->tensor, pre-allocated).

        dpred: gradient of the (B,T,V) predictions (batch-major), or time-major (T*B, V)
        when ``dpred_time_major``. dreg: (B,P) gradient added to every alphas[:, t]
        (the fused regulariser). dalphas: (B,T,P) gradient of the alphas output
        (generic autograd path). ``need``: names whose gradient is wanted (default: all
        present in ``grads``). ``denc``: (B,P,E) buffer receiving d(loss)/d(encoder_out) when
        the encoder is fine-tuned (models/encoder.py:112-121), else None. ``on_fc_grads``: called
        once the fc gradients are final, before the backward-through-time loop (data parallel: their
        all-reduce is issued there and runs beside the loop)."""
        dm, ws = st["dm"], st["ws"]
        B, T, L, P, A, D, M, V, E, X = dm.B, dm.T, dm.L, dm.P, dm.A, dm.D, dm.M, dm.V, dm.E, dm.X
        if st.get("dup", 1) > 1 and dalphas is not None:
            # the fused path's regulariser gradient arrives on the distinct rows (decoder_fn); a
            # per-position alphas gradient needs the full (B, P) layout. (denc on the distinct rows
            # is d(loss)/d(F x F map): the sum over each duplicate group, what the pool's backward
            # would form.)
            raise ValueError("capmi decoder: dalphas needs the full (non-deduplicated) features")
        enc, bt = st["enc"], st["bt"]
        need = set(grads) if need is None else set(need)
        gf = st.get("gflags", 0)
        W_ih = p["decode_step.weight_ih"]
        TB = T * B
        if dpred_time_major:
            ar = dict(a_r1=0, a_s2=0)
            lda_p = V
        else:
            ar = dict(a_r1=B, a_s2=V)
            lda_p = T * V
        if st["ragged"] and not dpred_time_major:
            # reference semantics: predictions of finished rows are constants (no gradient)
            dpred = dpred.clone()
            K.mask_rows_tb(dpred, st["bt_dev"], T, B, V, T * V, B, V)

        # ---- fc (:279): dHd = dpred W_fc ; dW_fc = dpred^T Hd ; db_fc = colsum(dpred)
        self._gemm_into(ws, ws.DHD, D, TB, D, V, dpred, lda_p, p["fc.weight"], D, AK, BKR, **ar, gf=gf)
        if "fc.weight" in need:
            self._gemm_into(ws, grads["fc.weight"], D, V, D, TB, dpred, lda_p, st["Hd"], D, AMM, BKR, **ar, gf=gf)
        if "fc.bias" in need:
            K.colsum(dpred, TB, V, V, grads["fc.bias"], ws.work)
        if on_fc_grads is not None:
            on_fc_grads()
        if st["dropout_p"] > 0:
            K.dropout(ws.DHD, ws.DHD.numel(), st["dropout_p"], st["seed"], ws.DHD, seed_dev=st["seed_dev"])

        # ---- backward through time
        s_dh = dm.s_dh
        S_dh = sum(s_dh)
        W_ih_awe = W_ih[:, M:]
        wf = p["attention.full_att.weight"]
        if denc is not None and getattr(ws, "DAWE", None) is None:
            ws.DAWE = torch.empty(T, B, E, device=enc.device, dtype=torch.float32)
            ws.DMEAN = torch.empty(B, E, device=enc.device, dtype=torch.float32)
        cur = 0
        if dm.fused:
            cur = self._bwd_loop_fused(p, st, dm, ws, enc, bt, dalphas, dreg, denc)
        for t in range(T - 1, -1, -1) if not dm.fused else ():
            K.lstm_cell_bwd(ws.DHD[t], ws.P_dh, S_dh if t < T - 1 else 0, B * D,
                            ws.DC[cur] if t < T - 1 else None, ws.ACT[t], ws.C[t], ws.C[t + 1], B, D, bt[t],
                            ws.DG[t], ws.DC[cur ^ 1])
            cur ^= 1
            K.gemm(K.problem(B, E, 4 * D, ws.DG[t], 4 * D, W_ih_awe, X, ws.P_dx, E, ksplit=dm.s_dx,
                             c_split_stride=B * E), AK, BKR, K.TILE_64, flags=gf)
            if dalphas is not None:
                dr, dr_ld = dalphas[:, t], T * P
            elif dreg is not None:
                dr, dr_ld = dreg, P
            else:
                dr, dr_ld = None, 0
            if dm.fused_att:
                K.att_bwd_fused(ws.P_dx, dm.s_dx, B * E, ws.GATE[t], ws.AWE[t], ws.DGP[t],
                                ws.DAWE[t] if denc is not None else None, enc, st["alphas"][:, t], T * P, dr, dr_ld,
                                ws.ATT_ENC, ws.AD[t], wf, B, P, A, E, bt[t], ws.DE[t], ws.DAD[t])
            else:
                K.att_ctx_bwd(ws.P_dx, dm.s_dx, B * E, ws.GATE[t], ws.AWE[t], enc, B, P, E, ws.DGP[t], ws.DALPHA,
                              dawe_out=ws.DAWE[t] if denc is not None else None)
                K.att_score_bwd(ws.DALPHA, dr, dr_ld, st["alphas"][:, t], T * P, ws.ATT_ENC, ws.AD[t], wf, B, P,
                                A, bt[t], ws.DE[t], ws.DAD[t])
            o1, o2 = s_dh[0] * B * D, (s_dh[0] + s_dh[1]) * B * D
            K.gemm([K.problem(B, D, 4 * D, ws.DG[t], 4 * D, p["decode_step.weight_hh"], D, ws.P_dh, D,
                              ksplit=s_dh[0], c_split_stride=B * D),
                    K.problem(B, D, E, ws.DGP[t], E, p["f_beta.weight"], D, ws.P_dh.view(-1)[o1:], D,
                              ksplit=s_dh[1], c_split_stride=B * D),
                    K.problem(B, D, A, ws.DAD[t], A, p["attention.dec_att.weight"], D,
                              ws.P_dh.view(-1)[o2:], D, ksplit=s_dh[2], c_split_stride=B * D)],
                   AK, BKR, K.TILE_64, flags=gf)
        # dh0 / dc0 -> h_lin / c_lin (:162-163)
        if not dm.fused:  # (the fused loop's last launch wrote DH0)
            K.splitk_reduce(ws.P_dh, S_dh, B * D, B, D, D, ws.DH0, D)
        dc0 = ws.DC[cur]
        for nm, dd in (("h_lin", ws.DH0), ("c_lin", dc0)):
            if nm + ".weight" in need:
                K.gemm(K.problem(D, E, B, dd, D, ws.mean, E, grads[nm + ".weight"], E), AMM, BKR, K.TILE_128, flags=gf)
            if nm + ".bias" in need:
                K.colsum(dd, B, D, D, grads[nm + ".bias"], ws.work)

        # ---- hoisted weight gradients over all t
        Hprev = ws.H[:T]
        if "decode_step.weight_ih" in need:
            self._gemm_into(ws, grads["decode_step.weight_ih"], X, 4 * D, X, TB, ws.DG, 4 * D, ws.X, X, AMM, BKR, gf=gf)
        if "decode_step.weight_hh" in need:
            self._gemm_into(ws, grads["decode_step.weight_hh"], D, 4 * D, D, TB, ws.DG, 4 * D, Hprev, D, AMM, BKR, gf=gf)
        if "decode_step.bias_ih" in need or "decode_step.bias_hh" in need:
            tgt = grads.get("decode_step.bias_ih", grads.get("decode_step.bias_hh"))
            K.colsum(ws.DG, TB, 4 * D, 4 * D, tgt, ws.work)
            for nm in ("decode_step.bias_ih", "decode_step.bias_hh"):
                if nm in need and grads[nm] is not tgt:
                    grads[nm].copy_(tgt)
        if "f_beta.weight" in need:
            self._gemm_into(ws, grads["f_beta.weight"], D, E, D, TB, ws.DGP, E, Hprev, D, AMM, BKR, gf=gf)
        if "f_beta.bias" in need:
            K.colsum(ws.DGP, TB, E, E, grads["f_beta.bias"], ws.work)
        if "attention.dec_att.weight" in need:
            self._gemm_into(ws, grads["attention.dec_att.weight"], D, A, D, TB, ws.DAD, A, Hprev, D, AMM, BKR, gf=gf)
        if "attention.dec_att.bias" in need:
            K.colsum(ws.DAD, TB, A, A, grads["attention.dec_att.bias"], ws.work)
        # d(att_enc) summed over t, full_att grads (:56-57), then enc_att grads (:54)
        nblk = K.att_enc_grad(ws.DE, ws.ATT_ENC, ws.AD, wf, T, B, P, A, ws.DATT, ws.WF_PART, ws.BF_PART)
        if "attention.full_att.weight" in need:
            K.colsum(ws.WF_PART, nblk, A, A, grads["attention.full_att.weight"], ws.work)
        if "attention.full_att.bias" in need:
            K.colsum(ws.BF_PART, nblk, 1, 1, grads["attention.full_att.bias"], ws.work)
        if "attention.enc_att.weight" in need:
            self._gemm_into(ws, grads["attention.enc_att.weight"], E, A, E, B * P, ws.DATT, A, enc, E, AMM, BKR, gf=gf)
        if "attention.enc_att.bias" in need:
            K.colsum(ws.DATT, B * P, A, A, grads["attention.enc_att.bias"], ws.work)
        # d(encoder_out): init mean (:161) + context sums (:59-60) + enc_att (:54)
        if denc is not None:
            K.gemm([K.problem(B, E, D, ws.DH0, D, p["h_lin.weight"], E, ws.DMEAN, E)], AK, BKR, K.TILE_64, flags=gf)
            K.gemm([K.problem(B, E, D, dc0, D, p["c_lin.weight"], E, ws.DMEAN, E, beta=1.0)], AK, BKR, K.TILE_64, flags=gf)
            K.att_enc_dinput(st["alphas"], T * P, ws.DAWE, ws.DMEAN, B, T, P, E, denc)
            self._gemm_into(ws, denc, E, B * P, E, A, ws.DATT, A, p["attention.enc_att.weight"], E, AK, BKR,
                            beta=1.0, gf=gf)
        # embedding (only when fine-tuned, Q8): dX_emb = DG W_ih[:, :M] -> scatter-add by token
        if "embedding.weight" in need and not st["dense_emb"]:
            demb = grads["embedding.weight"]
            demb.zero_()
            dxe = ws.scratch[:TB * M].view(TB, M)
            K.gemm(K.problem(TB, M, 4 * D, ws.DG, 4 * D, W_ih, X, dxe, M), AK, BKR, K.TILE_128, flags=gf)
            K.embed_scatter_add(dxe, M, st["caps"], B, L, T, st["bt_dev"], M, demb)
