"""Tile A/B for the decoder's hoisted weight-gradient GEMMs (batch 64, T = 24, k-major operands:
CAPMI_A_MMAJOR x CAPMI_B_KROWS, decoder_core.py _gemm_into), each tile vs TILE_AUTO.

python tools/dec_dw_ab.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_MMAJOR, CAPMI_B_KROWS  # noqa: E402

TB, BP = 64 * 24, 64 * 196
SHAPES = {"fc": (8100, 512, TB), "W_ih": (2048, 2560, TB), "W_hh": (2048, 512, TB), "f_beta": (2048, 512, TB),
          "dec_att": (512, 512, TB), "enc_att": (512, 2048, BP)}


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    dev = "cuda"
    ws = K.gemm_workspace(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    tiles = {"auto": K.TILE_AUTO, "128": K.TILE_128, "64": K.TILE_64, "128x64": K.TILE_128x64}
    for name, (M, N, Kd) in SHAPES.items():
        a = torch.rand(Kd, M, device=dev, generator=g) - 0.5
        b = torch.rand(Kd, N, device=dev, generator=g) - 0.5
        line = f"{name} M={M} N={N} K={Kd}:"
        for tn, t in tiles.items():
            out = torch.empty(M, N, device=dev)
            prob = K.problem(M, N, Kd, a, M, b, N, out, N)
            us = timeit(lambda: K.gemm_sk(prob, CAPMI_A_MMAJOR, ws, t, CAPMI_B_KROWS))
            plan = K.gemm_sk_plan(prob, CAPMI_A_MMAJOR, t, CAPMI_B_KROWS)
            line += f" {tn}{plan[:3]} {us:.1f}us {2.0 * M * N * Kd / us / 1e6:.1f}TF |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
