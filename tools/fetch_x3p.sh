#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of the x3p layer3 3x3 conv under schedule knobs (one PMC pass each)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for knob in "" "CAPMI_SK_GROUPS=1" "CAPMI_X3P_ORDER=col" "CAPMI_SK_HYBRID=0"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/fx/${knob:-default}_$C
    env $knob timeout -s KILL 60 rocprofv3 --pmc $C -d $d -o pmc -- python $R/tools/gemm_one.py --shape ${SHAPE:-l3c2} --reps 5 --x3p > /dev/null 2>&1 || exit 1
    python - $d $C <<'PY' >> $R/gpurun_out/fx_table.txt
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
v = [(r[0], r[1]) for r in c.execute("select value, duration from counters_collection where kernel_name like '%x3p%'")]
print(sys.argv[1].split("/")[-1], sys.argv[2], "KB/launch %.0f" % (sum(x for x, _ in v) / len(v)), "us %.1f" % (sum(d for _, d in v) / len(v) / 1e3))
PY
    rm -rf $d
  done
done
