"""Relative L2 error vs fp64 of the conv-shaped GEMM forms on ReLU'd-normal A (the encoder's conv
inputs) and normal B: native fp32 MFMA, gemm_x3 (in-kernel A split), x3p (both pre-split),
split-staged (both split in-kernel). python tools/x3_err.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "image-captioning-with-different-decoders_amd"))
from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_GEMM_SPLIT3  # noqa: E402


def main():
    dev = "cuda"
    ws = K.gemm_workspace(dev)
    for M, N, Kd in ((12544, 256, 2304), (12544, 1024, 256), (3136, 512, 4608)):
        g = torch.Generator().manual_seed(M + N + Kd)
        A = torch.relu(torch.randn(M, Kd, generator=g, dtype=torch.float64))
        B = torch.randn(N, Kd, generator=g, dtype=torch.float64) * (2.0 / Kd) ** 0.5
        ref = A @ B.T
        Af, Bf = A.float().to(dev), B.float().to(dev)
        out = torch.empty(M, N, device=dev)
        errs = {}

        def err():
            torch.cuda.synchronize()
            return float((out.double().cpu() - ref).norm() / ref.norm())
        K.gemm_sk(K.problem(M, N, Kd, Af, Kd, Bf, Kd, out, N), 0, ws)
        errs["fp32 MFMA"] = err()
        B3 = torch.empty(3 * N * Kd, device=dev, dtype=torch.bfloat16)
        K.split3_bf16(Bf, B3)
        K.gemm_x3(K.problem(M, N, Kd, Af, Kd, B3, Kd, out, N), 0, ws)
        errs["gemm_x3"] = err()
        A3 = torch.empty(3 * M * Kd, device=dev, dtype=torch.bfloat16)
        K.split3_bf16(Af, A3)
        K.gemm_x3p(K.problem(M, N, Kd, A3, Kd, B3, Kd, out, N), 0, ws)
        errs["x3p"] = err()
        K.gemm_sk(K.problem(M, N, Kd, Af, Kd, Bf, Kd, out, N), 0, ws, flags=CAPMI_GEMM_SPLIT3)
        errs["split-staged"] = err()
        # the fp32 CPU path (torch matmul in fp32) for scale
        errs["cpu fp32"] = float(((A.float() @ B.float().T).double() - ref).norm() / ref.norm())
        print(f"M={M} N={N} K={Kd}: " + ", ".join(f"{k} {v:.3g}" for k, v in errs.items()))


if __name__ == "__main__":
    main()
