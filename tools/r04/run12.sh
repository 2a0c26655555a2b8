#!/bin/bash
# round 4: x3p l3c2 pricing -- full-chip data-parallel (batch 167: 256 tiles) against the 98-tile grid, and the
# timing-only builds (no DMA / no barrier / zero-size descriptors) under stream-K and data-parallel grids
G="python -u tools/gemm_one.py --shape l3c2 --x3p --reps 50"
o=gpurun_out/x3p_price.txt
tools/gpu_steps.sh \
 "60|dp98|CAPMI_SK_OFF=1 $G > gpurun_out/p_dp98.txt" \
 "60|dp256|CAPMI_SK_OFF=1 $G --batch 167 > gpurun_out/p_dp256.txt" \
 "60|sk256|$G --batch 167 > gpurun_out/p_sk256.txt" \
 "60|sk64|$G > gpurun_out/p_sk64.txt" \
 "60|s1|CAPMI_LIB=ab/x3p_skip1.so $G > gpurun_out/p_s1.txt" \
 "60|s1dp|CAPMI_SK_OFF=1 CAPMI_LIB=ab/x3p_skip1.so $G > gpurun_out/p_s1dp.txt" \
 "60|s4|CAPMI_LIB=ab/x3p_skip4.so $G > gpurun_out/p_s4.txt" \
 "60|s4dp|CAPMI_SK_OFF=1 CAPMI_LIB=ab/x3p_skip4.so $G > gpurun_out/p_s4dp.txt" \
 "60|p3|CAPMI_LIB=ab/x3p_price3.so $G > gpurun_out/p_p3.txt" \
 "60|p3dp|CAPMI_SK_OFF=1 CAPMI_LIB=ab/x3p_price3.so $G > gpurun_out/p_p3dp.txt"
