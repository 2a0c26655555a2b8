"""Tile A/B for the fine-tune weight-gradient GEMMs (batch 64): dW[Cout, (kh, kw, ci)] =
dY[r, Cout]^T x im2col(relu(bn(y)))[r, (kh, kw, ci)] (CAPMI_A_MMAJOR x CAPMI_B_CONV_NHWC with the
BN prologue), the launch FineTuneRunner.backward makes for conv2 / conv3 / downsample, under each
tile (stream-K where it balances) vs TILE_AUTO.

python tools/wgrad_tile_ab.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_MMAJOR, CAPMI_B_CONV_NHWC  # noqa: E402

B = 64
# name: (Cin, H, Cout, k, stride) of the forward conv
SHAPES = {"l2c2": (128, 28, 128, 3, 1), "l3c2": (256, 14, 256, 3, 1), "l4c2": (512, 7, 512, 3, 1),
          "l2c3": (128, 28, 512, 1, 1), "l3c3": (256, 14, 1024, 1, 1), "l4c3": (512, 7, 2048, 1, 1)}


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
    for name, (ci, H, co, k, s) in SHAPES.items():
        Ho = (H + 2 * (k // 2) - k) // s + 1
        r = B * Ho * Ho
        dy = torch.rand(r, co, device=dev, generator=g) - 0.5
        y = torch.rand(B, H, H, ci, device=dev, generator=g) - 0.5
        sc = torch.rand(ci, device=dev, generator=g) + 0.5
        sh = torch.rand(ci, device=dev, generator=g) - 0.5
        geo = dict(N=B, H=H, W=H, Cin=ci, KH=k, KW=k, stride=s, pad=k // 2, Ho=Ho, Wo=Ho)
        N = ci * k * k
        ref = None
        line = f"{name} wgrad M={co} N={N} K={r}:"
        for tn, t in tiles.items():
            out = torch.empty(co, N, device=dev)
            prob = K.problem(co, N, r, dy, co, y, 0, out, N, conv=geo, in_scale=sc, in_shift=sh)
            us = timeit(lambda: K.gemm_sk(prob, CAPMI_A_MMAJOR, ws, t, CAPMI_B_CONV_NHWC))
            if ref is None:
                ref = out.clone()
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            plan = K.gemm_sk_plan(prob, CAPMI_A_MMAJOR, t, CAPMI_B_CONV_NHWC)
            line += f" {tn}{plan[:3]} {us:.1f}us {2.0 * co * N * r / us / 1e6:.1f}TF e{err:.0e} |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
