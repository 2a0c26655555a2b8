"""Per-shape time of the x3 conv kernels on the ResNet-101 encoder's unique conv shapes at batch 64:
gemm_x3 (A split while staging), x3d (A fp32 split in-kernel, B by LDS-DMA), x3p (+ its split pass).
python tools/r03/conv_ab.py [--reps 20] [--arms x3,x3d,x3p] [--only l3]  (CAPMI_LIB=<so>: another build)
Prints one markdown row per shape (us per launch, TF/s of the best arm) and the per-forward total of
the routed choice (capmi.resnet.EncoderRunner._conv's rule) and of the best arm."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from x3_ab import conv_shapes  # noqa: E402


def routed(tag, rows, Cin, Cout, k, st, pro):
    """The kernel EncoderRunner._conv picks for this shape in the x3 mode (resnet.py)."""
    kd = k * k * Cin
    in_ss = pro
    if kd == 64 and k == 1 and st == 1 and Cout in (64, 128, 256) and os.environ.get("CAPMI_X3S", "1") != "0":
        return "x3s"
    if Cin % 32 == 0 and kd % 32 == 0 and (st == 2 or (k == 1 and not in_ss and Cin == 2 * Cout)
                                           or rows <= 3136 or (k == 1 and in_ss and Cout == 4 * Cin)):
        return "x3d"  # (round 4 rule)
    if in_ss and Cout >= 128 and Cin % 32 == 0 and kd >= 128 and rows >= 12544:
        return "x3p"
    return "x3"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--arms", default="x3,x3d,x3p,x3s")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    arms_on = a.arms.split(",")
    dev = "cuda"
    ws = K.gemm_workspace(dev)
    tot_r, tot_b = 0.0, 0.0
    print(f"lib: {os.environ.get('CAPMI_LIB', 'in-tree')}")
    print("| conv | n | M | N | K | " + " | ".join(f"{x} us" for x in arms_on) + " | routed | best TF/s |")
    print("|---|---:|---:|---:|---:|" + "---:|" * len(arms_on) + "---|---:|")
    for (tag, N, H, Cin, Cout, k, st, pro), cnt in conv_shapes().items():
        if a.only and not tag.startswith(a.only):
            continue
        pad = k // 2
        Ho = (H + 2 * pad - k) // st + 1
        rows, Kd = N * Ho * Ho, k * k * Cin
        x = torch.rand(N * H * H * Cin, device=dev) * 2 - 0.5
        w = torch.randn(Cout, Kd, device=dev) * (2.0 / Kd) ** 0.5
        sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1
        stats = torch.zeros(2 * K.stat_tiles(rows) * Cout, device=dev)
        out = torch.empty(rows, Cout, device=dev)
        geo = dict(N=N, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=st, pad=pad, Ho=Ho, Wo=Ho)
        dense = k == 1 and st == 1 and not pro
        kw = dict(stats=stats)
        if not dense:
            kw.update(conv=geo, in_scale=sc if pro else None, in_shift=sh if pro else None)
        mode = 0 if dense else 2
        fns = {}
        if "x3" in arms_on:
            w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
            K.split3_bf16(w, w3)
            p3 = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w3, Kd, out, Cout, **kw)
            fns["x3"] = lambda: K.gemm_x3(p3, mode, ws)
        w3s = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(w, w3s)
        w3d = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, Cin).contiguous(), w3d)
        if "x3d" in arms_on and Cin % 32 == 0:
            if k == 1 and st == 1:  # 1x1: dense rows, the prologue per k = channel (round 3)
                pd = K.problem(rows, Cout, Kd, x, Cin, w3d, Kd, out, Cout, stats=stats,
                               in_scale=sc if pro else None, in_shift=sh if pro else None)
                fns["x3d"] = lambda: K.gemm_x3d(pd, 0, ws)
            else:
                pd = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w3d, Kd, out, Cout, **kw)
                fns["x3d"] = lambda: K.gemm_x3d(pd, mode, ws)
        if "x3s" in arms_on and Kd == 64 and k == 1 and st == 1 and Cout in (64, 128, 256):
            ps = K.problem(rows, Cout, Kd, x, Cin if dense else 0, w3s, Kd, out, Cout, **kw)
            fns["x3s"] = lambda: K.gemm_x3s(ps, mode)
        if "x3p" in arms_on and Cin % 32 == 0 and Kd >= 128:
            xp = torch.empty(3 * x.numel(), device=dev, dtype=torch.bfloat16)
            if k == 1 and st == 1:
                pp, mp = K.problem(rows, Cout, Kd, xp, Cin, w3d, Kd, out, Cout, stats=stats), 0
            else:
                pp, mp = K.problem(rows, Cout, Kd, xp, 0, w3d, Kd, out, Cout, conv=geo, stats=stats), 2

            def x3p_fn():
                K.bn_relu_split3(x, sc if pro else None, sh if pro else None, N * H * H, Cin, xp)
                K.gemm_x3p(pp, mp, ws)
            fns["x3p"] = x3p_fn
        res = {}
        for name, fn in fns.items():
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
        K.sk_check([ws])
        r = routed(tag, rows, Cin, Cout, k, st, pro)
        best = min(res.values())
        tot_r += res.get(r, best) * cnt
        tot_b += best * cnt
        f = 2.0 * rows * Cout * Kd
        print(f"| {tag} | {cnt} | {rows} | {Cout} | {Kd} | " +
              " | ".join(f"{res[x]:.1f}" if x in res else "-" for x in arms_on) +
              f" | {r} | {f / best / 1e6:.1f} |", flush=True)
    print(f"\nper forward: routed {tot_r / 1e3:.3f} ms, best arm {tot_b / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
