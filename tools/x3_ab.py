"""Per-shape conv time: native fp32 MFMA kernel (gemm_sk, TILE_AUTO) vs the x3 split kernel, on the
ResNet-101 encoder's unique conv shapes at batch 64 (train-mode prologue where the encoder has one).
python tools/x3_ab.py [--reps 20]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_GEMM_SPLIT3  # noqa: E402


def conv_shapes(B=64):
    # (tag, N, H, Cin, Cout, k, stride, prologue)
    out = []
    h, cin = 56, 64
    for li, (n, w, s) in enumerate(zip((3, 4, 23, 3), (64, 128, 256, 512), (1, 2, 2, 2))):
        for b in range(n):
            st = s if b == 0 else 1
            ho = (h + 2 - 3) // st + 1
            out.append((f"l{li + 1} c1 1x1", B, h, cin, w, 1, 1, False))
            out.append((f"l{li + 1} c2 3x3/{st}", B, h, w, w, 3, st, True))
            out.append((f"l{li + 1} c3 1x1", B, ho, w, 4 * w, 1, 1, True))
            if b == 0:
                out.append((f"l{li + 1} ds 1x1/{st}", B, h, cin, 4 * w, 1, st, False))
            cin, h = 4 * w, ho
    uniq = {}
    for sh in out:
        uniq.setdefault(sh, 0)
        uniq[sh] += 1
    return uniq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    ws = K.gemm_workspace(dev)
    tot = {"native": 0.0, "x3": 0.0}
    print("| conv | n | M | N | K | native us | TF/s | x3 us | TF/s | speedup | x3 kernel |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|")
    for (tag, N, H, Cin, Cout, k, st, pro), cnt in conv_shapes().items():
        pad = k // 2
        Ho = (H + 2 * pad - k) // st + 1
        rows, Kd = N * Ho * Ho, k * k * Cin
        x = torch.randn(N * H * H * Cin, device=dev)
        w = torch.randn(Cout, Kd, device=dev) * (2.0 / Kd) ** 0.5
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(w, w3)
        sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1
        stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=dev)
        out = torch.empty(rows, Cout, device=dev)
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=st, pad=pad, Ho=Ho, Wo=Ho)
        dense = k == 1 and st == 1 and not pro
        kw = dict(stats=stats)
        if not dense:
            kw.update(conv=geo, in_scale=sc if pro else None, in_shift=sh if pro else None)
        mode = 0 if dense else 2
        pn = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w, Kd, out, Cout, **kw)
        p3 = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w3, Kd, out, Cout, **kw)
        res = {}
        arms = [("native", lambda: K.gemm_sk(pn, mode, ws)), ("x3", lambda: K.gemm_x3(p3, mode, ws)),
                ("nts", lambda: K.gemm_sk(pn, mode, ws, flags=CAPMI_GEMM_SPLIT3)),
                ("nts128", lambda: K.gemm_sk(pn, mode, ws, K.TILE_128x64, flags=CAPMI_GEMM_SPLIT3))]
        if Cin % 32 == 0:  # x3d: A fp32 split in-kernel (+ prologue), B pre-split in the x3p order, DMA
            w3d = torch.empty_like(w3)
            K.split3_bf16(K.conv_weight_order_x3p(w, k, k, Cin).contiguous(), w3d)
            pd = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w3d, Kd, out, Cout, **kw)
            arms.append(("x3d", lambda: K.gemm_x3d(pd, mode, ws)))
        if pro and Cout >= 128 and Cin % 32 == 0:  # x3p candidates: split pass + pre-split GEMM
            xp = torch.empty(3 * x.numel(), device=dev, dtype=torch.bfloat16)
            w3p = torch.empty_like(w3)
            K.split3_bf16(K.conv_weight_order_x3p(w, k, k, Cin).contiguous(), w3p)
            if k == 1 and st == 1:
                pp, mp = K.problem(rows, Cout, Kd, xp, Cin, w3p, Kd, out, Cout, stats=stats), 0
            else:
                pp, mp = K.problem(rows, Cout, Kd, xp, 0, w3p, Kd, out, Cout, conv=geo, stats=stats), 2
            arms.append(("split", lambda: K.bn_relu_split3(x, sc, sh, N * H * H, Cin, xp)))
            arms.append(("x3p", lambda: K.gemm_x3p(pp, mp, ws)))
        for name, fn in arms:
            for _ in range(3):
                fn()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s0.record()
            for _ in range(a.reps):
                fn()
            s1.record()
            torch.cuda.synchronize()
            res[name] = s0.elapsed_time(s1) / a.reps * 1e3
        best = min(res["x3"], res.get("x3p", 1e9) + res.get("split", 0))
        tot["native"] += res["native"] * cnt
        tot["x3"] += best * cnt
        K.sk_check([ws])
        f = 2.0 * rows * Cout * Kd
        x3p = (f" x3p {res['x3p']:.1f} us ({f / res['x3p'] / 1e6:.1f} TF/s) + split {res['split']:.1f} us"
               if "x3p" in res else "")
        print(f"| {tag} | {cnt} | {rows} | {Cout} | {Kd} | {res['native']:.1f} | {f / res['native'] / 1e6:.1f} | "
              f"{res['x3']:.1f} | {f / res['x3'] / 1e6:.1f} | {res['native'] / best:.2f} | "
              f"{K.gemm_x3_kernel_name(p3, mode)}{x3p} | split-staged 64x64 {res['nts']:.1f} us, 128x64 "
              f"{res['nts128']:.1f} us | x3d {res.get('x3d', float('nan')):.1f} us |")
    print(f"\nlayer1-4 convs per forward: native {tot['native'] / 1e3:.3f} ms, best x3 form {tot['x3'] / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
