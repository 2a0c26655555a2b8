"""A/B of the fine-tune's 3x3 conv weight gradient (dW = dY^T im2col(relu(bn1(y1))), three-term
split, CAPMI_B_CONV_NHWC with the BN prologue): stream-K (what the runner launches) against
data-parallel k-splits, whose XCD-aware block remap hands each XCD one k-chunk of every output
tile (the A / B rows of that chunk are then read into one L2 once instead of once per tile).
Each launch timed alone with HIP events; the split partials' sum is timed separately (torch).

python tools/wgrad_split_ab.py [--reps 30]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "image-captioning-with-different-decoders_amd"))
from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_GEMM_SPLIT3  # noqa: E402

AMM, BCONV = 1, 2


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    ws = K.gemm_workspace(dev)
    print("| layer (N=64) | M x N x K | stream-K us | best split (tile, ks) us | sum us | max rel diff |")
    print("|---|---|---:|---:|---:|---:|")
    for name, H, wd in (("layer2 3x3 s1", 28, 128), ("layer3 3x3 s1", 14, 256), ("layer4 3x3 s1", 7, 512)):
        N = 64
        rows = N * H * H
        M_, N_, K_ = wd, 9 * wd, rows
        dy = torch.randn(rows * wd, device=dev, generator=g)
        y1 = torch.randn(rows * wd, device=dev, generator=g)
        sc = torch.rand(wd, device=dev, generator=g) + 0.5
        sh = torch.randn(wd, device=dev, generator=g) * 0.1
        geo = dict(N=N, H=H, W=H, Cin=wd, KH=3, KW=3, stride=1, pad=1, Ho=H, Wo=H)
        ref = torch.empty(M_ * N_, device=dev)
        p0 = K.problem(M_, N_, K_, dy, wd, y1, 0, ref, N_, conv=geo, in_scale=sc, in_shift=sh)
        t_sk = timed(lambda: K.gemm_sk(p0, AMM, ws, K.TILE_AUTO, BCONV, flags=CAPMI_GEMM_SPLIT3), a.reps)
        best, allt = None, []
        for tile, tname in ((K.TILE_128, "128x128"), (K.TILE_128x64, "128x64"), (K.TILE_64, "64x64")):
            for ks in (2, 4, 7, 8, 14, 16):
                part = torch.empty(ks * M_ * N_, device=dev)
                p = K.problem(M_, N_, K_, dy, wd, y1, 0, part, N_, conv=geo, in_scale=sc, in_shift=sh, ksplit=ks,
                              c_split_stride=M_ * N_)
                try:
                    t = timed(lambda: K.gemm(p, AMM, BCONV, tile, flags=CAPMI_GEMM_SPLIT3), a.reps)
                except Exception as e:  # noqa: BLE001
                    print(f"  {name} {tname} ks={ks}: {e}")
                    break
                allt.append(f"{tname}/{ks}:{t:.0f}")
                if best is None or t < best[0]:
                    best = (t, tname, ks, part)
        t, tname, ks, part = best
        out = torch.empty(M_, N_, device=dev)
        t_sum = timed(lambda: torch.sum(part.view(ks, M_, N_), 0, out=out), a.reps)
        K.gemm_sk(p0, AMM, ws, K.TILE_AUTO, BCONV, flags=CAPMI_GEMM_SPLIT3)
        torch.sum(part.view(ks, M_, N_), 0, out=out)
        torch.cuda.synchronize()
        diff = float(((out.view(-1) - ref).abs().max() / ref.abs().max()))
        print(f"| {name} | {M_} x {N_} x {K_} | {t_sk:.1f} | {t:.1f} ({tname}, {ks}) | {t_sum:.1f} | {diff:.1e} |")
        print("  all splits (us): " + " ".join(allt))
    K.sk_check([ws])


if __name__ == "__main__":
    main()
