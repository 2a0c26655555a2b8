#!/bin/bash
# round 4: the bf16 GEMM's prefetch fence (loads of tile kt+2 kept ahead of the step's MFMAs) -- bf16 parity, then
# config 5 against the unfenced build (ab/bf_old.so), alternating
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python bench.py --no-cpu-baseline --no-roofline --config bert_attention"
O="CAPMI_LIB=$PWD/ab/bf_old.so"
tools/gpu_steps.sh \
 "300|t|$P tests -m gpu -k 'bf16'" \
 "120|n1|$B > gpurun_out/b24_n1.json" \
 "120|o1|$O $B > gpurun_out/b24_o1.json" \
 "120|n2|$B > gpurun_out/b24_n2.json" \
 "120|o2|$O $B > gpurun_out/b24_o2.json" \
 "60|g1|python -u tools/gemm_one.py --shape l3c3 --bf16io --nopro --reps 50 > gpurun_out/b24_g1.txt" \
 "60|g0|$O python -u tools/gemm_one.py --shape l3c3 --bf16io --nopro --reps 50 > gpurun_out/b24_g0.txt"
