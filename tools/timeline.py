"""Busy/idle accounting of a rocprofv3 --kernel-trace CSV: per queue, how much of the wall time
between the last N step markers (one marker kernel per training step) kernels were running, the
summed kernel time, and the largest kernel families.
python tools/timeline.py gpurun_out/tl/tl_kernel_trace.csv [--marker adam_clamp] [--steps 10]"""
import argparse
import collections
import csv


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="adam_clamp")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if r["Kind"] == "KERNEL_DISPATCH"]
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    marks = [r["e"] for r in rows if a.marker in r["Kernel_Name"]]
    t0, t1 = marks[-a.steps - 1], marks[-1]
    win = [r for r in rows if r["s"] >= t0 and r["e"] <= t1]
    wall = (t1 - t0) / 1e3
    print(f"window: {a.steps} steps, {wall / a.steps:.1f} us/step wall, {len(win) / a.steps:.0f} kernels/step")
    print(f"any queue busy: {union([(r['s'], r['e']) for r in win]) / 1e3 / a.steps:.1f} us/step")
    byq = collections.defaultdict(list)
    for r in win:
        byq[r["Queue_Id"]].append(r)
    for q, rs in sorted(byq.items()):
        busy = union([(r["s"], r["e"]) for r in rs]) / 1e3 / a.steps
        summ = sum(r["e"] - r["s"] for r in rs) / 1e3 / a.steps
        fam = collections.Counter()
        for r in rs:
            fam[r["Kernel_Name"].split("(")[0][:70]] += (r["e"] - r["s"]) / 1e3 / a.steps
        print(f"queue {q}: {len(rs) / a.steps:.0f} kernels/step, busy {busy:.1f} us/step, summed {summ:.1f}")
        for k, v in fam.most_common(12):
            print(f"    {v:8.1f} us  {k}")


if __name__ == "__main__":
    main()
