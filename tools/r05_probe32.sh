#!/bin/bash
# round 5, probe 32: config 5's under-filled bf16 grids (layer4: 100 tiles of 128x128 on 256 CUs) at 128x64 tiles
G="python tools/gemm_one.py --reps 50 --bf16io"
s=""
for sh in l4c2 l4c2s l4c1 l4c3 ds4 l3c2 l3c1; do s="$s $G --shape $sh --tile 3 && $G --shape $sh --tile 2 &&"; done
tools/gpu_steps.sh "300|bf16_t2|${s% &&}"
grep "us/launch" gpurun_out/bf16_t2.log
