#!/bin/bash
# round 4: x3cw per-slice cost -- workers = tiles (one whole tile each, no partials) at 98 and 256 tiles, and
# stream-K on 196 / 256 workers
G="python -u tools/gemm_one.py --shape l3c2 --x3c --reps 50"
tools/gpu_steps.sh \
 "60|w98|CAPMI_SK_CUS=98 $G > gpurun_out/w_98.txt" \
 "60|w196|CAPMI_SK_CUS=196 $G > gpurun_out/w_196.txt" \
 "60|w256|$G > gpurun_out/w_256.txt" \
 "60|w256b|$G --batch 167 > gpurun_out/w_b167.txt" \
 "60|w128b|CAPMI_SK_CUS=128 $G --batch 167 > gpurun_out/w_b167_128.txt" \
 "60|c1|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/w_l1c2.txt" || exit $?
CASES="l3c2:x3c l3c2:x3p" bash tools/r03/sq.sh
