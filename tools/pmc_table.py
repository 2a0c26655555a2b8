"""Per-kernel average SQ counters from the pmc_x3.sh passes (gpurun_out/pmcx3/*/...db), with
derived ratios: MFMA busy % of SIMD cycles, wave-cycle split (wait / issue-stall / active), LDS
bank-conflict share, instructions per wave."""
import glob
import sqlite3
import sys
from collections import defaultdict


def load(db):
    c = sqlite3.connect(db)
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    dur = defaultdict(float)
    for did, name, cn, v, d in c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
        if "gemm" not in name:
            continue
        k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        per[k][cn] += v
        if did not in n[k]:
            n[k].add(did)
            dur[k] += d
    return {k: ({c: v / len(n[k]) for c, v in p.items()}, dur[k] / len(n[k]) / 1e3) for k, p in per.items()}


def main(root="gpurun_out/pmcx3"):
    runs = defaultdict(dict)
    for db in glob.glob(f"{root}/*/**/*.db", recursive=True) + glob.glob(f"{root}/*/*.db"):
        tag = db.split("/")[len(root.split("/"))].rsplit("_p", 1)[0]
        for k, (p, us) in load(db).items():
            runs[(tag, k)].update(p)
            runs[(tag, k)]["us"] = us
    for (tag, k), p in sorted(runs.items()):
        cyc = p.get("GRBM_GUI_ACTIVE", 0) / 8  # per-XCD cycles
        mf = p.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / cyc if cyc else 0
        wc = p.get("SQ_WAVE_CYCLES", 1)
        print(f"{tag:14s} {k[:48]:48s} {p['us']:7.1f} us  mfma_busy {100 * mf:5.1f}%  wait {100 * p.get('SQ_WAIT_ANY', 0) / wc:5.1f}%"
              f" stall {100 * p.get('SQ_WAIT_INST_ANY', 0) / wc:5.1f}% active {100 * p.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1f}%"
              f" lds_conflict {100 * p.get('SQ_LDS_BANK_CONFLICT', 0) / max(p.get('SQ_LDS_IDX_ACTIVE', 1), 1):5.1f}%"
              f" valu {p.get('SQ_INSTS_VALU', 0):.3g} mfma {p.get('SQ_INSTS_MFMA', 0):.3g} lds {p.get('SQ_INSTS_LDS', 0):.3g}"
              f" salu {p.get('SQ_INSTS_SALU', 0):.3g}")


if __name__ == "__main__":
    main(*sys.argv[1:])
