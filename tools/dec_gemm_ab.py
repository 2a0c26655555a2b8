"""Per-GEMM A/B of the decoder's GEMMs at the bench shape: fp32 MFMA vs CAPMI_GEMM_SPLIT3 vs
CAPMI_GEMM_BF16, each launch timed alone (HIP events over repeated launches, one stream).

python tools/dec_gemm_ab.py [--B 64] [--P 49] [--reps 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "image-captioning-with-different-decoders_amd"))
from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_GEMM_BF16, CAPMI_GEMM_SPLIT3  # noqa: E402
from capmi.decoder_core import DecoderDims  # noqa: E402

AK, AMM, BW, BKR = 0, 1, 0, 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--P", type=int, default=49)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tile", type=int, default=None, help="force this tile on the hoisted (stream-K) GEMMs")
    a = ap.parse_args()
    B, T, P, A, D, M, V, E = a.B, 24, a.P, 512, 512, 512, 8100, 2048
    dm = DecoderDims(B, T, 25, P, A, D, M, V, E)
    X, TB = dm.X, T * B
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def buf(*s):
        return torch.rand(*s, device=dev, generator=g) * 2 - 1

    big = buf(8 * 1024 * 1024 * 4)  # operand pool (A / B views)
    out = torch.empty(4 * 1024 * 1024 * 8, device=dev)
    ws = K.gemm_workspace(dev)

    def prob(M_, N_, K_, lda, ldb, ldc, ks=1, off=0):
        return K.problem(M_, N_, K_, big, lda, big[16 * 1024 * 1024:], ldb, out[off:], ldc, ksplit=ks,
                         c_split_stride=M_ * N_ if ks > 1 else 0)

    s_a, s_g, s_hh = dm.s_h
    cases = [
        ("step f: [att_dec|f_beta|W_hh] h (grouped)", "dp", AK, BW, K.TILE_64,
         lambda: [prob(B, A, D, D, D, A, s_a), prob(B, E, D, D, D, E, s_g, 4 << 20), prob(B, 4 * D, D, D, D, 4 * D, s_hh, 8 << 20)]),
        ("step f: W_ih_awe x", "dp", AK, BW, K.TILE_64, lambda: [prob(B, 4 * D, E, X, X, 4 * D, dm.s_x)]),
        ("step b: d(x) = dG W_ih_awe", "dp", AK, BKR, K.TILE_64, lambda: [prob(B, E, 4 * D, 4 * D, X, E, dm.s_dx)]),
        ("step b: dh (grouped)", "dp", AK, BKR, K.TILE_64,
         lambda: [prob(B, D, 4 * D, 4 * D, D, D, dm.s_dh[0]), prob(B, D, E, E, D, D, dm.s_dh[1], 4 << 20),
                  prob(B, D, A, A, D, D, dm.s_dh[2], 8 << 20)]),
        ("att_enc = enc W_ea^T", "sk", AK, BW, K.TILE_AUTO, lambda: prob(B * P, A, E, E, E, A)),
        ("xemb = X W_ih_emb^T", "sk", AK, BW, K.TILE_AUTO, lambda: prob(TB, 4 * D, M, X, X, 4 * D)),
        ("fc fwd", "sk", AK, BW, K.TILE_AUTO, lambda: prob(TB, V, D, D, D, V)),
        ("fc dgrad", "sk", AK, BKR, K.TILE_AUTO, lambda: prob(TB, D, V, V, D, D)),
        ("dW fc", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(V, D, TB, V, D, D)),
        ("dW ih", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(4 * D, X, TB, 4 * D, X, X)),
        ("dW hh", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(4 * D, D, TB, 4 * D, D, D)),
        ("dW f_beta", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(E, D, TB, E, D, D)),
        ("dW dec_att", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(A, D, TB, A, D, D)),
        ("dW enc_att", "sk", AMM, BKR, K.TILE_AUTO, lambda: prob(A, E, B * P, A, E, E)),
    ]
    flags = [("fp32", 0), ("x3", CAPMI_GEMM_SPLIT3), ("bf16", CAPMI_GEMM_BF16)]
    print(f"| GEMM (B={B}, P={P}) | " + " | ".join(f"{n} us" for n, _ in flags) + " |")
    print("|---|" + "---:|" * len(flags))
    tot = [0.0] * len(flags)
    for name, kind, am, bm, tile, mk in cases:
        row = []
        for fi, (_, f) in enumerate(flags):
            p = mk()

            def launch():
                if kind == "dp":
                    K.gemm(p, am, bm, tile, flags=f)
                else:
                    K.gemm_sk(p, am, ws, tile if a.tile is None else a.tile, bm, flags=f)
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                launch()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            row.append(us)
            tot[fi] += us * (T if kind == "dp" else 1)
        print(f"| {name} | " + " | ".join(f"{u:.1f}" for u in row) + " |")
    K.sk_check([ws])
    print(f"\nper training step (per-step GEMMs x {T}): " + ", ".join(f"{n} {t / 1e3:.3f} ms" for (n, _), t in zip(flags, tot)))


if __name__ == "__main__":
    main()
