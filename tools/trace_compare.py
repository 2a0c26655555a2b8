"""Compare per-step kernel time of selected kernels between rocprofv3 kernel-trace databases.

python tools/trace_compare.py OLD.db NEW.db [--kernels-per-step 531] [--steps 5]
Takes the last `steps` steps (kernels-per-step dispatches each) of every database and prints,
per kernel-name prefix, the summed duration per step and the mean per launch."""
import argparse
import sqlite3
from collections import defaultdict


def per_step(db, kps, steps):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()[-kps * steps:]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for name, s, e in rows:
        k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        tot[k] += (e - s) / 1e3 / steps
        cnt[k] += 1
    return tot, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--kernels-per-step", type=int, default=531)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    res = [per_step(d, a.kernels_per_step, a.steps) for d in a.dbs]
    keys = sorted(res[-1][0], key=lambda k: -res[-1][0][k])
    print("| kernel | " + " | ".join(f"us/step [{i}]" for i in range(len(res))) + " |")
    print("|---|" + "---:|" * len(res))
    for k in keys[:30]:
        print(f"| `{k}` | " + " | ".join(f"{r[0].get(k, 0):.1f}" for r in res) + " |")
    print("| total | " + " | ".join(f"{sum(r[0].values()):.1f}" for r in res) + " |")


if __name__ == "__main__":
    main()
