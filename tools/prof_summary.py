"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd SQLite) into markdown.

python tools/prof_summary.py gpurun_out/prof/bench_results.db [--steps 5 --warmup 2] > profiles/x.md

Per kernel: calls, total/avg/min/max duration and share. With --steps/--warmup the
per-step view divides the totals by (steps + warmup) bench steps.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc"))
    tot = sum(r[2] for r in rows)
    nsteps = a.steps + a.warmup
    print(f"# rocprofv3 kernel summary: `{a.db}`\n")
    print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches"
          + (f" ({nsteps} bench steps -> {tot / 1e6 / nsteps:.3f} ms/step of kernel time)" if nsteps else ""))
    print("\n| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, n, s, avg, mn, mx in rows[:a.top]:
        short = name if len(name) < 90 else name[:87] + "..."
        print(f"| `{short}` | {n} | {s / 1e6:.3f} | {avg / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | "
              f"{100 * s / tot:.1f} |")


if __name__ == "__main__":
    main()
