"""In-graph cost of each per-timestep decoder kernel at the bench's shapes (B = 64, 49 distinct rows, A = D = 512,
E = 2048, x3 GEMMs): every call of one timestep (t = 0 forward, t = T-1 .. backward) captured n times back to back in
a HIP graph and replayed -- wall time per call, the figure a graph replay of the step pays (rocprofv3's per-kernel
durations add ~3-4 us of tracing to each). python tools/dec_kernels.py"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def per_call(fn, n=100, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def main():
    import gen
    from capmi import decoder_fn as DF
    from capmi import kernels as K
    from capmi._lib import CAPMI_A_KMAJOR as AK, CAPMI_B_KROWS as BKR, CAPMI_B_NMAJOR_W as BW
    from helpers import make_decoder, t
    dev = "cuda"
    B, L, V = 64, 25, 8100
    dec, _ = make_decoder(512, 512, 512, V, 5, dev)
    dec.set_compute_precision("fp32-x3")
    dec.train()
    dec.fine_tune_embeddings(False)
    enc = t(gen.encoder_features(5, B, P=49), dev).view(B, 7, 7, 2048)
    caps = t(gen.captions(5, B, L, V), dev)
    grads = {n: torch.zeros_like(q) for n, q in dec.named_parameters() if q.requires_grad}
    DF.fused_loss_and_grads(dec, enc, caps, [L] * B, 1.0, grads, dup=2)
    torch.cuda.synchronize()
    ws = next(iter(DF.CORE._ws.values()))
    dm_key = next(iter(DF.CORE._ws))
    from capmi.decoder_core import DecoderDims
    dm = DecoderDims(*dm_key[0])
    p = DF.decoder_params(dec)
    gf = DF.gemm_flags(dec)
    P, A, D, E, M, X, T = dm.P, dm.A, dm.D, dm.E, dm.M, dm.X, dm.T
    s_a, s_g, s_hh = dm.s_h
    encf = enc.reshape(B, P, E)
    alphas = torch.empty(B, T, P, device=dev)
    W_ih = p["decode_step.weight_ih"]
    h, tt = ws.H[0], 0
    calls = {
        "fwd h-GEMM (att_dec | f_beta | W_hh)": lambda: K.gemm(
            [K.problem(B, A, D, h, D, p["attention.dec_att.weight"], D, ws.P_ad, A, ksplit=s_a, c_split_stride=B * A),
             K.problem(B, E, D, h, D, p["f_beta.weight"], D, ws.P_gate, E, ksplit=s_g, c_split_stride=B * E),
             K.problem(B, 4 * D, D, h, D, p["decode_step.weight_hh"], D, ws.P_hh, 4 * D, ksplit=s_hh,
                       c_split_stride=B * 4 * D)], AK, BW, K.TILE_64, flags=gf),
        "fwd att_score": lambda: K.att_score_fwd(ws.ATT_ENC, ws.P_ad, s_a, B * A, p["attention.dec_att.bias"],
                                                 p["attention.full_att.weight"], p["attention.full_att.bias"], B, P, A,
                                                 ws.score, ws.AD[tt]),
        "fwd att_softmax_ctx": lambda: K.att_softmax_ctx_fwd(ws.score, encf, B, P, E, B, alphas[:, tt], T * P,
                                                             ws.AWE[tt], ws.P_gate, s_g, B * E, p["f_beta.bias"],
                                                             ws.GATE[tt], ws.X[tt, :, M:], X),
        "fwd x-GEMM (W_ih awe half)": lambda: K.gemm(
            K.problem(B, 4 * D, E, ws.X[tt, :, M:], X, W_ih[:, M:], X, ws.P_x, 4 * D, ksplit=dm.s_x,
                      c_split_stride=B * 4 * D), AK, BW, K.TILE_64, flags=gf),
        "fwd lstm_cell": lambda: K.lstm_cell_fwd(ws.P_x, dm.s_x, B * 4 * D, ws.XEMB[tt], ws.P_hh, s_hh, B * 4 * D,
                                                 ws.C[tt], B, D, ws.H[tt + 1], ws.C[tt + 1], ws.ACT[tt]),
        "bwd dx-GEMM": lambda: K.gemm(K.problem(B, E, 4 * D, ws.DG[tt], 4 * D, W_ih[:, M:], X, ws.P_dx, E,
                                                ksplit=dm.s_dx, c_split_stride=B * E), AK, BKR, K.TILE_64, flags=gf),
        "bwd dh-GEMM (grouped)": lambda: K.gemm(
            [K.problem(B, D, 4 * D, ws.DG[tt], 4 * D, p["decode_step.weight_hh"], D, ws.P_dh, D, ksplit=dm.s_dh[0],
                       c_split_stride=B * D),
             K.problem(B, D, E, ws.DGP[tt], E, p["f_beta.weight"], D, ws.P_dh.view(-1)[dm.s_dh[0] * B * D:], D,
                       ksplit=dm.s_dh[1], c_split_stride=B * D),
             K.problem(B, D, A, ws.DAD[tt], A, p["attention.dec_att.weight"], D,
                       ws.P_dh.view(-1)[(dm.s_dh[0] + dm.s_dh[1]) * B * D:], D, ksplit=dm.s_dh[2], c_split_stride=B * D)],
            AK, BKR, K.TILE_64, flags=gf),
        "bwd att_ctx": lambda: K.att_ctx_bwd(ws.P_dx, dm.s_dx, B * E, ws.GATE[tt], ws.AWE[tt], encf, B, P, E, ws.DGP[tt],
                                             ws.DALPHA),
        "bwd att_score": lambda: K.att_score_bwd(ws.DALPHA, None, 0, alphas[:, tt], T * P, ws.ATT_ENC, ws.AD[tt],
                                                 p["attention.full_att.weight"], B, P, A, B, ws.DE[tt], ws.DAD[tt]),
    }
    tot = 0.0
    for name, fn in calls.items():
        us = per_call(fn)
        tot += us
        print(f"{name:38s} {us:7.2f} us per call in a graph", flush=True)
    print(f"{'sum (one timestep, fwd + bwd, no lstm bwd)':38s} {tot:7.2f} us; x {T} = {tot * T / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
