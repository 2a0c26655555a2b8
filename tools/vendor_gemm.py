"""Yardstick: the vendor GEMM (torch.matmul -> hipBLASLt/rocBLAS, fp32 with TF32 off, and bf16) on
the dense GEMM shapes of the encoder convs at batch 64 (M = 64*Ho*Wo, N = Cout, K = Cin*k*k), to
compare with tools/gemm_one.py (our implicit-GEMM conv kernels, which also do im2col, the BN
prologue and the statistics epilogue)."""
import torch

SHAPES = {"l3c2": (12544, 256, 2304), "l3c3": (12544, 1024, 256), "l3c1": (12544, 256, 1024),
          "l2c2": (50176, 128, 1152), "l4c2": (3136, 512, 4608), "l1c2": (200704, 64, 576),
          "l1c3": (200704, 256, 64), "l4c3": (3136, 2048, 512)}


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    for name, (M, N, K) in SHAPES.items():
        for dt in (torch.float32, torch.bfloat16):
            a = torch.randn(M, K, device="cuda", dtype=dt)
            b = torch.randn(N, K, device="cuda", dtype=dt)
            c = torch.empty(M, N, device="cuda", dtype=dt)
            for _ in range(3):
                torch.matmul(a, b.t(), out=c)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(30):
                torch.matmul(a, b.t(), out=c)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / 30
            print(f"{name} {str(dt)[6:]}: M={M} N={N} K={K}: {us:.1f} us, {2.0 * M * N * K / us / 1e6:.1f} TFLOP/s",
                  flush=True)


if __name__ == "__main__":
    main()
