"""Calibration: sustained vendor (hipBLASLt via torch.matmul) bf16 / fp32 GEMM throughput on this
MI355X, i.e. the practical MFMA ceiling the x3 kernels are judged against.
python tools/vendor_peak.py"""
import torch


def bench(n, dtype, reps=20):
    a = torch.randn(n, n, device="cuda", dtype=dtype)
    b = torch.randn(n, n, device="cuda", dtype=dtype)
    for _ in range(3):
        a @ b
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        a @ b
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    return 2.0 * n ** 3 / us / 1e6


if __name__ == "__main__":
    torch.backends.cuda.matmul.allow_tf32 = False
    for n in (4096, 8192):
        print(f"n={n}: bf16 {bench(n, torch.bfloat16):.0f} TFLOP/s, fp32 {bench(n, torch.float32):.0f} TFLOP/s")
