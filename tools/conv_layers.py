"""Per-layer-kind conv GEMM throughput from a rocprofv3 kernel-trace database.

python tools/conv_layers.py gpurun_out/prof/bench_results.db [--batch 64]

Walks the last encoder forward in the trace (the launch order of capmi.resnet.EncoderRunner:
conv1, then per bottleneck conv1/conv2/conv3[/downsample]) and reports TFLOP/s per shape."""
import argparse
import sqlite3


def shapes(B, H=224):
    out = []
    h = (H + 6 - 7) // 2 + 1
    out.append(("conv1 7x7/2", B * h * h, 64, 147))
    h = (h + 2 - 3) // 2 + 1
    cin = 64
    for li, (n, w, s) in enumerate(zip((3, 4, 23, 3), (64, 128, 256, 512), (1, 2, 2, 2))):
        for b in range(n):
            st = s if b == 0 else 1
            ho = (h + 2 - 3) // st + 1
            out.append((f"l{li + 1} c1 1x1", B * h * h, w, cin))
            out.append((f"l{li + 1} c2 3x3/{st}", B * ho * ho, w, 9 * w))
            out.append((f"l{li + 1} c3 1x1", B * ho * ho, 4 * w, w))
            if b == 0:
                out.append((f"l{li + 1} ds 1x1/{st}", B * ho * ho, 4 * w, cin))
            cin, h = 4 * w, ho
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, duration from kernels order by start"))
    sh = shapes(a.batch)
    # conv1 follows the image re-layout kernel (or is the older NCHW-gather generic kernel)
    starts = [i for i, r in enumerate(rows) if "image_nhwc4" in r[0]]
    if starts:
        gem = [r for r in rows[starts[-1]:] if "gemm" in r[0]]
        convs = gem[:len(sh)]
    else:
        gem = [r for r in rows if "gemm" in r[0]]
        first = [i for i, r in enumerate(gem) if "3, 0" in r[0] and "gemm_kernel<" in r[0]]
        convs = gem[first[-1]:first[-1] + len(sh)]
    agg, tf, tt = {}, 0, 0
    for (tag, M, N, K), (name, d) in zip(sh, convs):
        f = 2 * M * N * K
        e = agg.setdefault(tag, [0, 0, 0, M, N, K, set()])
        e[0] += f
        e[1] += d
        e[2] += 1
        e[6].add(name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0])
        tf += f
        tt += d
    print(f"| layer / conv | n | M | N | K | ms | TFLOP/s | kernel |\n|---|---:|---:|---:|---:|---:|---:|---|")
    for k, (f, d, n, M, N, K, names) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"| {k} | {n} | {M} | {N} | {K} | {d / 1e6:.3f} | {f / d / 1e3:.1f} | {', '.join(sorted(names))} |")
    print(f"\nencoder convs: {tt / 1e6:.3f} ms, {tf / tt / 1e3:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
