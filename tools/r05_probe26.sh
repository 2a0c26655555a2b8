#!/bin/bash
# round 5, probe 26: x3p tile walk order (CAPMI_X3P_ORDER=col: an XCD group's tiles share one weight column block)
# at the current kernel: per-conv times, L2 hit rate, bench pair
G="python tools/gemm_one.py --reps 50 --x3p"
s=""
for sh in l3c2 l2c2 l3c2s l2c2s; do s="$s $G --shape $sh && CAPMI_X3P_ORDER=col $G --shape $sh &&"; done
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh "300|ord_alone|${s% &&}" \
  "120|ord_l2|mkdir -p gpurun_out/l2 && cd /tmp && export TMPDIR=/tmp && CAPMI_X3P_ORDER=col timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $R/gpurun_out/l2/l3c2col -o pmc -- python $R/tools/gemm_one.py --shape l3c2 --reps 5 --x3p > /dev/null 2>&1 && cd $R && python tools/pmc_l2.py gpurun_out/l2 && rm -rf gpurun_out/l2" \
  "200|ob1|$B" "200|oc1|CAPMI_X3P_ORDER=col $B" "200|ob2|$B" "200|oc2|CAPMI_X3P_ORDER=col $B"
for f in ob1 oc1 ob2 oc2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
