"""A/B on the fine-tune backward's plain GEMMs (batch 64): our capmi_gemm_sk launch as
FineTuneRunner.backward makes it vs the vendor GEMM (torch.mm -> hipBLASLt/rocBLAS, TF32 off).

  conv1.wgrad  dW[wd, Cin]   = dA1[r, wd]^T X[r, Cin]      (A_MMAJOR x B_KROWS)
  conv1.dgrad  dX[r, Cin]    = dA1[r, wd] W1[wd, Cin]      (A_KMAJOR x B_KROWS)
  conv3.dgrad  dA2[r, wd]    = dY3[r, Cout] W3[Cout, wd]   (A_KMAJOR x B_KROWS)

python tools/bwd_gemm_ab.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_B_KROWS, CAPMI_B_NMAJOR_W  # noqa: E402

B = 64
LAYERS = {"l2": (512, 128, 28), "l3": (1024, 256, 14), "l4": (2048, 512, 7)}  # Cin(=Cout), wd, H


def timeit(fn, reps=30):
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
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = "cuda"
    ws = K.gemm_workspace(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (C, wd, H) in LAYERS.items():
        r = B * H * H
        da = torch.rand(r, wd, device=dev, generator=g) - 0.5
        x = torch.rand(r, C, device=dev, generator=g) - 0.5
        w1 = torch.rand(wd, C, device=dev, generator=g) - 0.5
        dy3 = torch.rand(r, C, device=dev, generator=g) - 0.5
        w3 = torch.rand(C, wd, device=dev, generator=g) - 0.5
        cases = {
            "conv1.wgrad": (wd, C, r, lambda o: K.problem(wd, C, r, da, wd, x, C, o, C), CAPMI_A_MMAJOR,
                            lambda o: torch.mm(da.t(), x, out=o), (wd, C)),
            "conv1.dgrad": (r, C, wd, lambda o: K.problem(r, C, wd, da, wd, w1, C, o, C), CAPMI_A_KMAJOR,
                            lambda o: torch.mm(da, w1, out=o), (r, C)),
            "conv3.dgrad": (r, wd, C, lambda o: K.problem(r, wd, C, dy3, C, w3, wd, o, wd), CAPMI_A_KMAJOR,
                            lambda o: torch.mm(dy3, w3, out=o), (r, wd)),
        }
        for cname, (M, N, Kd, mk, amode, vend, shp) in cases.items():
            o1 = torch.empty(shp, device=dev)
            o2 = torch.empty(shp, device=dev)
            prob = mk(o1)
            ours = timeit(lambda: K.gemm_sk(prob, amode, ws, K.TILE_AUTO, CAPMI_B_KROWS))
            ven = timeit(lambda: vend(o2))
            err = ((o1 - o2).abs().max() / o2.abs().max()).item()
            plan = K.gemm_sk_plan(prob, amode, K.TILE_AUTO, CAPMI_B_KROWS, threads=True)
            f = 2.0 * M * N * Kd
            extra = ""
            if cname.endswith("wgrad"):
                for tn, t in (("64", K.TILE_64), ("128", K.TILE_128), ("128x64", K.TILE_128x64)):
                    us = timeit(lambda: K.gemm_sk(prob, amode, ws, t, CAPMI_B_KROWS))
                    extra += f" | {tn}: {us:.1f} us ({f / us / 1e6:.1f} TF/s)"
            if cname.endswith("dgrad"):
                # B = W[n][k]: the 1x1 weight transposed by conv_weight_pack_dgrad (CAPMI_B_NMAJOR_W)
                wsrc = w1 if cname == "conv1.dgrad" else w3
                wt = torch.empty(wsrc.shape[1], wsrc.shape[0], device=dev)
                K.conv_weight_pack_dgrad(wsrc.view(*wsrc.shape, 1, 1), wt)
                o3 = torch.empty(shp, device=dev)
                pt = K.problem(M, N, Kd, da if cname == "conv1.dgrad" else dy3, Kd, wt, Kd, o3, N)
                ourst = timeit(lambda: K.gemm_sk(pt, CAPMI_A_KMAJOR, ws, K.TILE_AUTO, CAPMI_B_NMAJOR_W))
                e3 = ((o3 - o2).abs().max() / o2.abs().max()).item()
                pl3 = K.gemm_sk_plan(pt, CAPMI_A_KMAJOR, K.TILE_AUTO, CAPMI_B_NMAJOR_W, threads=True)
                extra = f" | W^T {pl3}: {ourst:.1f} us ({f / ourst / 1e6:.1f} TF/s) relerr {e3:.1e}"
            print(f"{name} {cname}: M={M} N={N} K={Kd} plan={plan}: ours {ours:.1f} us ({f / ours / 1e6:.1f} TF/s)"
                  f" vendor {ven:.1f} us ({f / ven / 1e6:.1f} TF/s) relerr {err:.1e}{extra}", flush=True)


if __name__ == "__main__":
    main()
