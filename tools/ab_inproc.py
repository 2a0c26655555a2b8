"""Same-process A/B of library builds on single conv GEMM launches: every build is loaded side by side
(capmi._lib._load) and the builds take turns, `--rounds` times, on the same tensors, so clock and box drift
fall on all arms alike. Prints the median us per launch of each build per case, and whether each build's output
equals the first build's bit for bit.

python tools/ab_inproc.py --libs base,ab/ph2.so --cases "l3c2:--x3p l3c3:--x3d,--dense" [--reps 20 --rounds 7]
(base = the in-tree libcapmi.so; a case is a tools/gemm_one.py shape and its flags, commas for spaces)"""
import argparse
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_one import parser, setup  # noqa: E402
from capmi import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    names = a.libs.split(",")
    libs = {n: (_lib.lib if n == "base" else _lib._load(n)) for n in names}
    base = _lib.lib
    print("| case | " + " | ".join(os.path.basename(n) for n in names) + " |")
    print("|---|" + "---:|" * len(names))
    for case in a.cases.split():
        shape, _, flags = case.partition(":")
        g = parser().parse_args(["--shape", shape] + [f for f in flags.split(",") if f])
        run, M, N, Kd = setup(g)
        times = {n: [] for n in names}
        same = {}
        for n in names:
            _lib.lib = libs[n]
            run.out.fill_(float("nan"))
            run()
            torch.cuda.synchronize()
            same[n] = torch.equal(run.out, same[names[0]]) if n != names[0] else run.out.clone()
        same[names[0]] = True
        for _ in range(a.rounds):
            for n in names:
                _lib.lib = libs[n]
                run()  # warm this build's code object
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[n].append(s.elapsed_time(e) * 1e3 / a.reps)
        _lib.lib = base
        print(f"| {case} | " + " | ".join(f"{st.median(times[n]):.1f}{'' if same[n] else ' (DIFFERS)'}" for n in names) + " |", flush=True)


if __name__ == "__main__":
    main()
