"""Times the encoder's elementwise passes alone at their batch-64 shapes (bn_add_relu, bn_finalize, bn_relu_split3)
against a plain torch copy of the same bytes: HBM / Infinity-Cache rate check. Usage: python tools/eltwise_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
from capmi import kernels as K  # noqa: E402


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


dev = "cuda"
for (M, C) in ((200704, 256), (50176, 512), (12544, 1024), (3136, 2048), (12544, 256), (50176, 128)):
    y = torch.rand(M, C, device=dev)
    r = torch.rand(M, C, device=dev)
    o = torch.empty(M, C, device=dev)
    s = torch.rand(C, device=dev)
    b = torch.rand(C, device=dev)
    mb = M * C * 4 / 1e6
    t1 = timeit(lambda: K.bn_add_relu(y, s, b, r, o, M, C))
    t2 = timeit(lambda: torch.add(y, r, out=o))
    # rotate over 8 distinct buffers: cold-ish (beyond the L2s, maybe in the Infinity Cache)
    ys = [torch.rand(M, C, device=dev) for _ in range(4)]
    it = iter(range(10 ** 9))
    t3 = timeit(lambda: K.bn_add_relu(ys[next(it) % 4], s, b, r, o, M, C))
    stats = torch.rand(2 * K.stat_tiles(M) * C, device=dev)
    g, be, rm, rv = (torch.rand(C, device=dev) for _ in range(4))
    sc, sh = torch.empty(C, device=dev), torch.empty(C, device=dev)
    work = torch.zeros(K.bn_work_doubles(2048), device=dev, dtype=torch.float64)
    t4 = timeit(lambda: K.bn_finalize(stats, K.stat_tiles(M), C, M, g, be, rm, rv, 0.1, 1e-5, sc, sh, work))
    xp = torch.empty(3 * M * C, device=dev, dtype=torch.bfloat16)
    t5 = timeit(lambda: K.bn_relu_split3(y, s, b, M, C, xp))
    print(f"M={M:6d} C={C:4d} {mb:6.1f} MB/tensor | bn_add_relu {t1:7.2f} us ({3 * mb / t1:5.2f} TB/s) rot {t3:7.2f} "
          f"| torch add {t2:7.2f} us ({3 * mb / t2:5.2f} TB/s) | bn_finalize {t4:6.2f} us | split3 {t5:7.2f} us "
          f"({5 * mb / 2 / t5:5.2f} TB/s)", flush=True)
