#!/bin/bash
# A/B of library builds: tools/ab_libs.sh lib1.so lib2.so ... -> gpurun_out/ab_libs.txt
# single conv GEMMs (tools/gemm_one.py) then a short bench per build (no CPU baseline)
set -o pipefail
out=gpurun_out/ab_libs.txt; : > $out
for v in "$@"; do
  for sh in l3c2 l3c3 l3c1 l1c2 l1c3; do
    CAPMI_LIB=$v timeout -k 10 60 python tools/gemm_one.py --shape $sh --reps 100 2>&1 | grep TFLOP | sed "s|^|$v |" >> $out || exit 1
  done
done
for v in "$@"; do
  CAPMI_LIB=$v timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_bench.log') if l.startswith('{')][-1]); print('$v', 'bench', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['conv_family']['conv_ms_per_step'])" >> $out
done
