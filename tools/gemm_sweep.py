"""GEMM / implicit-GEMM conv throughput sweep over the tile shapes (GPU only).

python tools/gemm_sweep.py [--reps 20]
Prints TFLOP/s per (shape, tile) on random operands (random data: the chip clocks differently
on zeros). Shapes: a 4096^3 calibration GEMM and every distinct ResNet-101 conv at batch 64.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_CONV_NHWC, CAPMI_A_KMAJOR, CAPMI_B_NMAJOR_W  # noqa: E402

TILES = {0: "128x128", 1: "64x64", 2: "128x64", 3: "auto"}
SK_TILES = {1: "64x64 SK", 2: "128x64 SK"}


def time_launch(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--scan", action="store_true", help="occupancy scan: N=256, K=2304, M varied")
    a = ap.parse_args()
    if a.scan:
        return scan(a)
    dev = "cuda"
    N = a.batch
    # (name, Cin, H, W, Cout, k, stride, prologue)
    convs = [("l1 c1", 64, 56, 56, 64, 1, 1, False), ("l1 c2", 64, 56, 56, 64, 3, 1, True),
             ("l1 c3", 64, 56, 56, 256, 1, 1, True), ("l2 c1", 256, 56, 56, 128, 1, 1, False),
             ("l2 c2", 128, 28, 28, 128, 3, 1, True), ("l2 c3", 128, 28, 28, 512, 1, 1, True),
             ("l3 c1", 512, 28, 28, 256, 1, 1, False), ("l3 c1'", 1024, 14, 14, 256, 1, 1, False), ("l3 c2", 256, 14, 14, 256, 3, 1, True),
             ("l3 c3", 256, 14, 14, 1024, 1, 1, True), ("l4 c1", 1024, 14, 14, 512, 1, 1, False),
             ("l4 c1'", 2048, 7, 7, 512, 1, 1, False),
             ("l4 c2", 512, 7, 7, 512, 3, 1, True), ("l4 c3", 512, 7, 7, 2048, 1, 1, True)]
    g = torch.Generator(device=dev).manual_seed(0)
    print("| shape | M | N | K | " + " | ".join(list(TILES.values()) + list(SK_TILES.values())) + " |")
    print("|---|---:|---:|---:|" + "---:|" * (len(TILES) + len(SK_TILES)))
    ws = K.gemm_workspace(dev)
    S = 4096
    A = torch.rand(S, S, device=dev, generator=g) - 0.5
    B = torch.rand(S, S, device=dev, generator=g) - 0.5
    C = torch.empty(S, S, device=dev)
    res = []
    for t in TILES:
        sec = time_launch(lambda: K.gemm(K.problem(S, S, S, A, S, B, S, C, S), CAPMI_A_KMAJOR,
                                         CAPMI_B_NMAJOR_W, t), a.reps)
        res.append(2.0 * S ** 3 / sec / 1e12)
    print(f"| gemm 4096^3 | {S} | {S} | {S} | " + " | ".join(f"{r:.1f}" for r in res) + " |")
    del A, B, C
    for name, ci, H, W, co, k, st, pro in convs:
        pd = k // 2
        Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        M, Kd = N * Ho * Wo, ci * k * k
        x = torch.rand(N, H, W, ci, device=dev, generator=g) - 0.5
        w = torch.rand(co, Kd, device=dev, generator=g) - 0.5
        y = torch.empty(M, co, device=dev)
        stats = torch.empty(K.stat_tiles(M, 1) * co * 2 + 64, device=dev)
        sc = torch.rand(ci, device=dev, generator=g) + 0.5
        sh = torch.rand(ci, device=dev, generator=g) - 0.5
        geo = dict(N=N, H=H, W=W, Cin=ci, KH=k, KW=k, stride=st, pad=pd, Ho=Ho, Wo=Wo)
        res = []
        for t in TILES:
            if k == 1 and not pro:
                prob = K.problem(M, co, Kd, x, ci, w, Kd, y, co, stats=stats)
                mode = CAPMI_A_KMAJOR
            else:
                prob = K.problem(M, co, Kd, x, 0, w, Kd, y, co, conv=geo, stats=stats,
                                 in_scale=sc if pro else None, in_shift=sh if pro else None)
                mode = CAPMI_A_CONV_NHWC
            sec = time_launch(lambda: K.gemm(prob, mode, CAPMI_B_NMAJOR_W, t), a.reps)
            res.append(2.0 * M * co * Kd / sec / 1e12)
        for t in SK_TILES:
            sec = time_launch(lambda: K.gemm_sk(prob, mode, ws, t), a.reps)
            res.append(2.0 * M * co * Kd / sec / 1e12)
        print(f"| {name} {k}x{k} | {M} | {co} | {Kd} | " + " | ".join(f"{r:.1f}" for r in res) + " |")
        del x, w, y


def scan(a):
    """Time vs tile count at fixed per-tile work: flat time => per-block latency bound,
    linear => throughput bound (then wave quantisation costs what the tile counts say)."""
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    Nn, Kd = 256, 2304
    w = torch.rand(Nn, Kd, device=dev, generator=g) - 0.5
    print("| M | tiles64 | us 64x64 | us 128x64 | us 128x128 |")
    print("|---:|---:|---:|---:|---:|")
    for M in (1024, 4096, 8192, 12544, 16384, 20480, 24576, 32768, 49152):
        x = torch.rand(M, Kd, device=dev, generator=g) - 0.5
        y = torch.empty(M, Nn, device=dev)
        r = []
        for t in (1, 2, 0):
            prob = K.problem(M, Nn, Kd, x, Kd, w, Kd, y, Nn)
            r.append(time_launch(lambda: K.gemm(prob, CAPMI_A_KMAJOR, CAPMI_B_NMAJOR_W, t), a.reps) * 1e6)
        print(f"| {M} | {M // 64 * 4} | " + " | ".join(f"{v:.1f}" for v in r) + " |")


if __name__ == "__main__":
    main()
