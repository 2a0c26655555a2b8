"""Per-kernel cost floor on the chip: a HIP graph of n back-to-back tiny kernels (capmi counter_add), replayed,
wall time per kernel; and the same with a 4 MB store per kernel (bn_add_relu on a small tensor), to separate the
dispatch / completion floor from the work. python tools/launch_floor.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
from capmi import kernels as K  # noqa: E402


def per_kernel(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


c = torch.zeros(1, dtype=torch.int64, device="cuda")
print(f"counter_add (1 thread): {per_kernel(lambda: K.counter_add(c, 1)):.2f} us per kernel in a graph")
for rows in (64, 4096, 65536):
    y = torch.rand(rows, 64, device="cuda")
    r = torch.rand(rows, 64, device="cuda")
    o = torch.empty(rows, 64, device="cuda")
    s_ = torch.rand(64, device="cuda")
    b_ = torch.rand(64, device="cuda")
    t = per_kernel(lambda: K.bn_add_relu(y, s_, b_, r, o, rows, 64))
    print(f"bn_add_relu {rows}x64 ({rows * 64 * 4 / 1e6:.2f} MB out): {t:.2f} us per kernel in a graph")
