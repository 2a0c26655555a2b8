#!/bin/bash
# bf16-IO conv GEMM timings per ResNet shape for library builds: tools/ab_bf16.sh lib1.so lib2.so ...
set -o pipefail
out=gpurun_out/ab_bf16.txt; : > $out
for v in "$@"; do
  for sh in l3c2 l3c3 l3c1 l1c2 l2c2 l4c2; do
    CAPMI_LIB=$v timeout -k 10 60 python tools/gemm_one.py --shape $sh --reps 50 --bf16io 2>&1 | grep TFLOP | sed "s|^|$v |" >> $out || exit 1
  done
done
