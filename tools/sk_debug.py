"""Stream-K GEMM diagnostics (GPU): repeated launches vs the data-parallel kernel and fp64.

python tools/sk_debug.py
For each shape: max |SK - fp64| per launch, whether launches agree bitwise, the number of flags
left non-zero and the spin-timeout word after each launch.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402


def main():
    dev = "cuda"
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = torch.Generator().manual_seed(0)
    for M, N, Kd, tile in [(64, 64, 4608, 1), (64, 64, 256, 1), (3136, 256, 2304, 1), (3136, 256, 2304, 2),
                           (200, 130, 300, 1), (12544, 256, 1024, 1)]:
        X = torch.rand(M, Kd, generator=g, dtype=torch.float64) * 2 - 1
        W = torch.rand(N, Kd, generator=g, dtype=torch.float64) * 2 - 1
        ref = X @ W.T
        Xd, Wd = X.float().to(dev), W.float().to(dev)
        C = torch.empty(M, N, device=dev)
        ws = K.gemm_workspace(dev)
        nflags = cus * 4 + 1
        K.gemm(K.problem(M, N, Kd, Xd, Kd, Wd, Kd, C, N), 0, 0, tile)
        torch.cuda.synchronize()
        dp_err = float((C.double().cpu() - ref).abs().max())
        outs = []
        for it in range(4):
            C.fill_(float("nan"))
            K.gemm_sk(K.problem(M, N, Kd, Xd, Kd, Wd, Kd, C, N), 0, ws, tile)
            torch.cuda.synchronize()
            Cc = C.double().cpu()
            err = (Cc - ref).abs()
            fl = ws[:nflags].cpu()
            bad = (err > 1e-3).nonzero()
            print(f"M={M} N={N} K={Kd} tile={tile} launch {it}: max err {float(err.max()):.3g} "
                  f"(dp {dp_err:.3g}) nan={int(torch.isnan(Cc).sum())} flags_left={int((fl[:-1] != 0).sum())} "
                  f"timeout={int(fl[-1])} bad={bad.shape[0]}"
                  + (f" first bad rc={bad[0].tolist()} last={bad[-1].tolist()}" if bad.shape[0] else ""), flush=True)
            outs.append(Cc)
        print("  bitwise equal across launches:", all(torch.equal(outs[0], o) for o in outs[1:]), flush=True)


if __name__ == "__main__":
    main()
