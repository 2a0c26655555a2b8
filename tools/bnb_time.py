"""BN backward passes of the fine-tune encoder (encoder_bwd.hip: bn_bwd_reduce + its finalize, bn_bwd_apply) timed
per shape, every library build side by side in one process (capmi._lib._load), outputs compared with the first
build's (apply bit for bit when the coefficients are the same; the reduce's coefficients to 1e-5 relative).
python tools/bnb_time.py --libs base,ab/bnb0.so [--rounds 5]"""
import argparse
import os
import statistics as st
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402
from capmi import _lib  # noqa: E402
from capmi import kernels as K  # noqa: E402

# (rows, C, mode): layer2 / layer3 / layer4 in-block BN (RELU_Y) and the bottleneck tails (RELU_OUT), batch 64
SHAPES = [(50176, 128, 0), (12544, 256, 0), (3136, 512, 0), (12544, 1024, 1), (3136, 2048, 1), (50176, 512, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    names = a.libs.split(",")
    libs = {n: (_lib.lib if n == "base" else _lib._load(n)) for n in names}
    base = _lib.lib
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(3)
    work = torch.zeros(K.bnb_work_floats(2048), device=dev)
    print("| rows x C (mode) | pass | " + " | ".join(os.path.basename(n) for n in names) + " | GB/s (first) |")
    print("|---|---|" + "---:|" * len(names) + "---:|")
    for rows, C, mode in SHAPES:
        d = torch.randn(rows, C, device=dev, generator=g)
        y = torch.randn(rows, C, device=dev, generator=g)
        out = torch.relu(torch.randn(rows, C, device=dev, generator=g)) if mode == 1 else None
        sc = torch.rand(C, device=dev, generator=g) + 0.5
        sh = torch.rand(C, device=dev, generator=g) - 0.5
        gamma = torch.rand(C, device=dev, generator=g) + 0.5
        mean = y.mean(0)
        var = y.var(0, unbiased=False)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        coef = torch.empty(4 * C, device=dev)
        dy = torch.empty(rows, C, device=dev)
        scs, shs = (sc, sh) if mode == 0 else (None, None)
        red = lambda: K.bn_bwd_reduce(mode, d, y, out, scs, shs, gamma, mean, var, 1e-5, rows, C, dg, db,  # noqa: E731
                                      coef, work)
        app = lambda: K.bn_bwd_apply(mode, d, y, out, scs, shs, coef, rows, C, dy)  # noqa: E731
        res = {}
        for n in names:
            _lib.lib = libs[n]
            red()
            c0 = coef.clone()
            app()
            torch.cuda.synchronize()
            res[n] = (c0, dy.clone())
        t = {(n, p): [] for n in names for p in ("reduce", "apply")}
        for _ in range(a.rounds):
            for n in names:
                _lib.lib = libs[n]
                for p, fn in (("reduce", red), ("apply", app)):
                    fn()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.reps):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    t[(n, p)].append(s.elapsed_time(e) * 1e3 / a.reps)
        _lib.lib = base
        c_ref, _ = res[names[0]]
        for p, nbytes in (("reduce", (2 + (mode == 1)) * rows * C * 4), ("apply", (3 + (mode == 1)) * rows * C * 4)):
            cells = []
            for n in names:
                cn, dn = res[n]
                ok = torch.allclose(cn, c_ref, rtol=1e-5, atol=1e-7) if p == "reduce" else \
                    (torch.equal(dn, res[names[0]][1]) or not torch.equal(cn, c_ref))
                cells.append(f"{st.median(t[(n, p)]):.2f}{'' if ok else ' (DIFFERS)'}")
            us0 = st.median(t[(names[0], p)])
            print(f"| {rows} x {C} ({mode}) | {p} | " + " | ".join(cells) + f" | {nbytes / us0 / 1e3:.0f} |", flush=True)


if __name__ == "__main__":
    main()
