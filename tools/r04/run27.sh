#!/bin/bash
# round 4 diagnostic: the clock x3p's workgroups hold (s_memtime / s_memrealtime x 100 MHz, diagnostic build
# ab/x3p_clk.so) on l3c2 -- 98 tiles data-parallel, 256 tiles data-parallel (batch 167), stream-K on 256 workers
G="python -u tools/gemm_one.py --shape l3c2 --x3p --reps 4000"
L="CAPMI_LIB=$PWD/ab/x3p_clk.so"
tools/gpu_steps.sh \
 "120|k98|$L CAPMI_SK_OFF=1 $G > gpurun_out/clk_dp98.txt" \
 "120|k256|$L CAPMI_SK_OFF=1 $G --batch 167 > gpurun_out/clk_dp256.txt" \
 "120|ksk|$L $G > gpurun_out/clk_sk.txt"
