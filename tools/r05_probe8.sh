#!/bin/bash
# round 5, probe 8: the unfenced sc1 stream-K hand-off of the one-workgroup-per-CU x3 kernels (in-tree) against
# the round-4 fenced form (ab/fenced.so): hand-off stress test, parity, same-process A/B, bench pairs
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CASES="l3c2:--x3p l2c2:--x3p l3c3:--x3d,--dense l4c3:--x3d,--dense l4c2:--x3d l3c2s:--x3d ds3:--x3d l4c1:--x3"
B="python bench.py --no-cpu-baseline"
tools/gpu_steps.sh \
  "400|par8|$T tests/test_gpu_sk_handoff.py tests/test_gpu_x3.py -k 'handoff or x3p or x3d or encoder_x3_matches or beta'" \
  "600|ab8|python tools/ab_inproc.py --libs base,ab/fenced.so --cases '$CASES' --reps 20 --rounds 5" \
  "200|b8_base1|$B > gpurun_out/b8_base1.json" \
  "200|b8_f1|CAPMI_LIB=ab/fenced.so $B > gpurun_out/b8_f1.json" \
  "200|b8_base2|$B > gpurun_out/b8_base2.json" \
  "200|b8_f2|CAPMI_LIB=ab/fenced.so $B > gpurun_out/b8_f2.json"
