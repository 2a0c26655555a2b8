#!/bin/bash
# round 5, probe 19: config 5's bf16 GEMM with one LDS stage and four workgroups per CU (st1) vs two stages and two
# (base), at 128x128 (tile 3 = auto) and 128x64 (tile 2)
c=""
for sh in l3c3 l2c3 l4c3 l3c1 l1c3 l3c2; do c="$c $sh:--bf16io $sh:--bf16io,--tile,2"; done
tools/gpu_steps.sh "240|bf16_st1|python tools/ab_inproc.py --libs base,ab/st1.so --cases \"${c# }\" --rounds 5"
