#!/bin/bash
# round 5, probe 23: config 5's 3x3 bf16 convs per shape, data-parallel (default) vs stream-K (CAPMI_BF16_SK=1)
G="python tools/gemm_one.py --reps 50 --bf16io"
s=""
for sh in l2c2 l3c2 l4c2 l2c2s l3c2s l4c2s l4c1 l4c3 ds4; do
  s="$s CAPMI_BF16_SK=0 $G --shape $sh && CAPMI_BF16_SK=1 $G --shape $sh &&"
done
tools/gpu_steps.sh "300|bf16_sk|${s% &&}"
