"""Beam-search captioning on the capmi kernels.

Restates ``attention_caption_image_beam_search`` (gen_captions.py:16-131 of the reference): one
image, k beams treated as a batch of k, per step the soft attention, the f_beta gate, the
LSTMCell and the vocabulary projection, then log_softmax + top-k over the (beams x V) scores and
the bookkeeping of finished beams. The arithmetic of a step runs on the same HIP kernels as the
training forward (grouped h-GEMM, fused ReLU score, softmax + context + gate, LSTM pointwise);
``enc_att(encoder_out)`` is computed once per image (the reference recomputes it every step,
Q5). The selection logic (top-k over at most k*V scores, beam reordering) is a few tiny torch
ops on the device, as in the reference.
"""
import torch

from . import kernels as K
from ._lib import CAPMI_A_KMAJOR as AK, CAPMI_B_NMAJOR_W as BW


class BeamSearch:
    def __init__(self, decoder, beam_size):
        self.dec = decoder
        self.k = int(beam_size)
        if self.k < 1:
            raise ValueError("beam_size must be >= 1")

    def _params(self):
        d = self.dec
        return dict(W_ea=d.attention.enc_att.weight, b_ea=d.attention.enc_att.bias,
                    W_da=d.attention.dec_att.weight, b_da=d.attention.dec_att.bias,
                    wf=d.attention.full_att.weight.view(-1), bf=d.attention.full_att.bias,
                    W_ih=d.decode_step.weight_ih, W_hh=d.decode_step.weight_hh,
                    b_ih=d.decode_step.bias_ih, b_hh=d.decode_step.bias_hh,
                    W_h=d.h_lin.weight, b_h=d.h_lin.bias, W_c=d.c_lin.weight, b_c=d.c_lin.bias,
                    W_fb=d.f_beta.weight, b_fb=d.f_beta.bias, W_fc=d.fc.weight, b_fc=d.fc.bias,
                    emb=d.embedding.weight)

    @torch.no_grad()
    def search(self, encoder_out, start_idx, end_idx, max_steps=50, return_all=False):
        """encoder_out: (1, 14, 14, E) or (1, P, E) features of ONE image. Returns
        (sequence list[int], alphas list (steps, P), finished bool) like the reference
        (failure: ([start, end], [], False)); with ``return_all`` also (every finished sequence,
        their scores)."""
        if self.dec.use_bert:
            raise NotImplementedError("beam search with BERT features (the reference notes it fails too)")
        p = self._params()
        dev = encoder_out.device
        E = encoder_out.size(-1)
        enc1 = encoder_out.reshape(1, -1, E).contiguous().float()
        P = enc1.size(1)
        k = self.k
        A, D = p["W_ea"].shape[0], p["W_hh"].shape[1]
        M, V = p["emb"].shape[1], p["W_fc"].shape[0]
        X = M + E
        f = dict(device=dev, dtype=torch.float32)
        # per image: att_enc once, init state (gen_captions.py:57; models/attention.py:151-164)
        att1 = torch.empty(P, A, **f)
        K.gemm(K.problem(P, A, E, enc1, E, p["W_ea"], E, att1, A, bias=p["b_ea"]), AK, BW, K.TILE_64)
        mean = torch.empty(1, E, **f)
        K.mean_rows(enc1, 1, P, E, mean)
        h = torch.empty(k, D, **f)
        c = torch.empty(k, D, **f)
        K.gemm([K.problem(1, D, E, mean, E, p["W_h"], E, h, D, bias=p["b_h"]),
                K.problem(1, D, E, mean, E, p["W_c"], E, c, D, bias=p["b_c"])], AK, BW, K.TILE_64)
        h[1:] = h[0]
        c[1:] = c[0]
        # beams of one image share its features: expanded once
        encK = enc1.expand(k, P, E).contiguous()
        attK = att1.unsqueeze(0).expand(k, P, A).contiguous()
        xin = torch.empty(k, X, **f)
        p_ad, p_gate = torch.empty(k, A, **f), torch.empty(k, E, **f)
        p_hh, p_x = torch.empty(k, 4 * D, **f), torch.empty(k, 4 * D, **f)
        e = torch.empty(k, P, **f)
        alpha, awe, gate = torch.empty(k, P, **f), torch.empty(k, E, **f), torch.empty(k, E, **f)
        act, h2, c2 = torch.empty(k, 4 * D, **f), torch.empty(k, D, **f), torch.empty(k, D, **f)
        scores = torch.empty(k, V, **f)

        prev = torch.full((k, 1), start_idx, dtype=torch.int64, device=dev)
        seqs = prev.clone()
        top = torch.zeros(k, 1, **f)
        seq_alpha = torch.ones(k, 1, P, **f)
        done_seqs, done_alpha, done_scores = [], [], []
        s, step, ended = k, 1, False
        while True:
            # embeddings (gen_captions.py:64) -> x[:, :M]; attention + gate -> x[:, M:]
            K.embed_gather(p["emb"], prev, s, 1, 1, xin, X)
            K.gemm([K.problem(s, A, D, h, D, p["W_da"], D, p_ad, A),
                    K.problem(s, E, D, h, D, p["W_fb"], D, p_gate, E),
                    K.problem(s, 4 * D, D, h, D, p["W_hh"], D, p_hh, 4 * D)], AK, BW, K.TILE_64)
            K.att_score_fwd(attK, p_ad, 1, 0, p["b_da"], p["wf"], p["bf"], s, P, A, e)
            K.att_softmax_ctx_fwd(e, encK, s, P, E, s, alpha, P, awe, p_gate, 1, 0, p["b_fb"], gate,
                                  xin[:, M:], X)
            K.gemm(K.problem(s, 4 * D, X, xin, X, p["W_ih"], X, p_x, 4 * D, bias=p["b_ih"], bias2=p["b_hh"]),
                   AK, BW, K.TILE_64)
            K.lstm_cell_fwd(p_x, 1, 0, None, p_hh, 1, 0, c, s, D, h2, c2, act)
            K.gemm(K.problem(s, V, D, h2, D, p["W_fc"], D, scores, V, bias=p["b_fc"]), AK, BW, K.TILE_64)
            # selection (gen_captions.py:74-117)
            lp = torch.log_softmax(scores[:s], dim=1) + top.expand(s, V)
            if step == 1:
                top_s, top_w = lp[0].topk(s, 0, True, True)
            else:
                top_s, top_w = lp.view(-1).topk(s, 0, True, True)
            prev_i = torch.div(top_w, V, rounding_mode="floor")
            next_w = top_w % V
            seqs = torch.cat([seqs[prev_i], next_w.unsqueeze(1)], dim=1)
            seq_alpha = torch.cat([seq_alpha[prev_i], alpha[:s][prev_i].unsqueeze(1)], dim=1)
            nw = next_w.tolist()
            inc = [i for i, w in enumerate(nw) if w != end_idx]
            com = sorted(set(range(len(nw))) - set(inc))
            if com:
                ended = True
                done_seqs.extend(seqs[com].tolist())
                done_alpha.extend(seq_alpha[com].tolist())
                done_scores.extend(top_s[com].tolist())
            s -= len(com)
            if s == 0:
                break
            seqs, seq_alpha = seqs[inc], seq_alpha[inc]
            top = top_s[inc].unsqueeze(1)
            sel = prev_i[inc]
            h[:s] = h2[:len(nw)][sel]
            c[:s] = c2[:len(nw)][sel]
            prev = next_w[inc].unsqueeze(1).contiguous()
            if step > max_steps:
                break
            step += 1
        extra = ((done_seqs, done_scores),) if return_all else ()
        if not ended:
            return ([start_idx, end_idx], [], False) + extra
        best = done_scores.index(max(done_scores))
        al = done_alpha[best]
        if encoder_out.dim() == 4:  # (steps+1, 14, 14) like the reference's seqs_alpha
            hh, ww = encoder_out.size(1), encoder_out.size(2)
            al = [[row[i * ww:(i + 1) * ww] for i in range(hh)] for row in al]
        return (done_seqs[best], al, True) + extra
