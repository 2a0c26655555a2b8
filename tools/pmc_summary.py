"""Aggregate rocprofv3 --pmc counters per kernel name from a rocpd database.

python tools/pmc_summary.py gpurun_out/pmc1/pmc_results.db [--filter gemm]
Prints per kernel: dispatches, summed duration and summed counter values (counters_collection
already holds the per-dispatch totals), plus derived ratios when the inputs are present:
  wait%  = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue-stall% = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 4 SIMD * 256 CU / 8 XCD-share),
  HBM bytes = 2 * FETCH_SIZE (KB; gfx950 reports half of wide streaming reads) + WRITE_SIZE."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
    per = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    dur = defaultdict(float)
    for did, name, cn, v, d in rows:
        if a.filter and a.filter not in name:
            continue
        k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        per[k][cn] += v
        if did not in seen[k]:
            seen[k].add(did)
            dur[k] += d
    for k in sorted(per, key=lambda x: -dur[x]):
        p = per[k]
        line = f"{k:70s} n={len(seen[k]):4d} {dur[k] / 1e6:8.3f} ms"
        if "SQ_WAVE_CYCLES" in p and p["SQ_WAVE_CYCLES"]:
            wc = p["SQ_WAVE_CYCLES"]
            line += f" wait {100 * p.get('SQ_WAIT_ANY', 0) / wc:5.1f}% stall {100 * p.get('SQ_WAIT_INST_ANY', 0) / wc:5.1f}%"
            line += f" active {100 * p.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1f}%"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in p and "GRBM_GUI_ACTIVE" in p and p["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE summed over 8 XCDs; MFMA busy summed over all SIMDs (1024)
            util = p["SQ_VALU_MFMA_BUSY_CYCLES"] / (p["GRBM_GUI_ACTIVE"] / 8 * 1024)
            line += f" mfma_util {100 * util:5.1f}%"
        if "FETCH_SIZE" in p:
            line += f" fetch(x2) {2 * p['FETCH_SIZE'] / 1024 / len(seen[k]):9.1f} MB/launch"
        if "WRITE_SIZE" in p:
            line += f" write {p['WRITE_SIZE'] / 1024 / len(seen[k]):9.1f} MB/launch"
        print(line)


if __name__ == "__main__":
    main()
