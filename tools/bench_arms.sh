#!/bin/bash
# Same-box A/B of environment arms on the bench line (no roofline pass, no CPU baseline: ~5 s per run), the arms
# interleaved ROUNDS times so box drift spreads over all of them; prints img/s per run and the mean per arm.
#   ARMS="base= wgs512=CAPMI_DEC_WGS=512 f1=CAPMI_DEC_FUSED=1" ROUNDS=3 [BENCH_ARGS=--config ...] tools/bench_arms.sh
ROUNDS=${ROUNDS:-3}
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for arm in ${ARMS:-base=}; do
    name=${arm%%=*}; envs=${arm#*=}; envs=${envs//,/ }
    out=$(env $envs timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline $BENCH_ARGS) || exit 1
    v=$(python -c "import json,sys;print(json.loads(sys.argv[1])['value'])" "$out")
    echo "$name $v" | tee -a gpurun_out/bench_arms.txt
  done
done
python - <<'PY'
import collections
d = collections.defaultdict(list)
for line in open("gpurun_out/bench_arms.txt"):
    n, v = line.split()
    d[n].append(float(v))
for n, vs in d.items():
    print(f"mean {n:12s} {sum(vs) / len(vs):9.2f} img/s over {len(vs)}")
PY
