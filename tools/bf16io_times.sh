#!/bin/bash
# bf16-IO conv GEMM timings per ResNet shape (batch 64) -> gpurun_out/bf16io_times.txt
set -o pipefail
out=gpurun_out/bf16io_times.txt; : > $out
for sh in l3c2 l3c3 l3c1 l1c2 l1c3 l2c2 l4c2; do
  timeout -k 10 60 python tools/gemm_one.py --shape $sh --reps 50 --bf16io 2>&1 | grep TFLOP | sed "s|^|bf16io |" >> $out || exit 1
done
