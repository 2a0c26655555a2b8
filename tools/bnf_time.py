"""Time capmi_bn_finalize alone on the encoder's BN shapes at batch 64 (slices of 64 rows, channels)."""
import sys

import torch

sys.path.insert(0, "image-captioning-with-different-decoders_amd")
from capmi import kernels as K  # noqa: E402

SHAPES = [(196, 256), (196, 1024), (49, 512), (49, 2048), (784, 128), (784, 512), (3136, 64), (3136, 256)]


def main():
    dev = "cuda"
    work = torch.zeros(K.bn_work_doubles(2048), device=dev, dtype=torch.float64)
    for tiles, C in SHAPES:
        st = torch.rand(tiles, C, 2, device=dev)
        g, b = torch.rand(C, device=dev), torch.rand(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        sc, sh = torch.empty(C, device=dev), torch.empty(C, device=dev)
        run = lambda: K.bn_finalize(st, tiles, C, tiles * 64, g, b, rm, rv, 0.1, 1e-5, sc, sh, work)  # noqa: E731
        run()
        torch.cuda.synchronize()
        # replayed from a HIP graph: the per-call host cost of ctypes would otherwise dominate
        gr = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            with torch.cuda.graph(gr, stream=side):
                for _ in range(100):
                    run()
        gr.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            gr.replay()
        e.record()
        torch.cuda.synchronize()
        print(f"bn_finalize tiles={tiles} C={C}: {s.elapsed_time(e) * 1e3 / 500:.2f} us", flush=True)


if __name__ == "__main__":
    main()
