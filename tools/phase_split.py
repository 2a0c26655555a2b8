"""Split one training step of a rocprofv3 kernel trace into encoder / decoder-forward /
loss / decoder-backward / optimizer phases and list the top kernels of each.

python tools/phase_split.py gpurun_out/prof/bench_results.db"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select name, duration, start, end from kernels order by start"))
    # a step starts at conv1 (the image re-layout kernel that feeds it, or the older NCHW gather)
    starts = [i for i, r in enumerate(rows)
              if "image_nhwc4" in r[0] or "gemm_kernel<128, 128, 64, 64, 3" in r[0]] + [len(rows)]
    # the last complete training step: a segment between two conv1 launches that contains Adam
    segs = [(a, b) for a, b in zip(starts, starts[1:]) if any("adam_clamp" in r[0] for r in rows[a:b])]
    i0, i1 = segs[-1]
    step = rows[i0:i1]
    wall = step[-1][3] - step[0][2]
    phase = "encoder"
    tot = defaultdict(float)
    per = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for name, d, s, e in step:
        if phase == "encoder" and "embed_gather" in name:
            phase = "decoder_fwd"
        elif phase == "decoder_fwd" and "ce_fwd_bwd" in name:
            phase = "loss"
        elif phase == "loss" and "gemm" in name:
            phase = "decoder_bwd"
        elif "adam_clamp" in name:
            phase = "optimizer"
        tot[phase] += d
        per[phase][short(name)][0] += 1
        per[phase][short(name)][1] += d
    print(f"one step: {len(step)} kernels, kernel time {sum(tot.values()) / 1e6:.3f} ms, wall {wall / 1e6:.3f} ms")
    for ph in ("encoder", "decoder_fwd", "loss", "decoder_bwd", "optimizer"):
        print(f"\n## {ph}: {tot[ph] / 1e6:.3f} ms")
        for k, (n, d) in sorted(per[ph].items(), key=lambda x: -x[1][1])[:8]:
            print(f"  {d / 1e3:9.1f} us  x{n:<4d} {k}")


if __name__ == "__main__":
    main()
