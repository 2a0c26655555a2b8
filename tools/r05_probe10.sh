#!/bin/bash
# round 5, probe 10: gemm_x3 with the mid-tile barrier and the split of tile kt + 2 behind it (X3_PHASE); x3p vs
# x3d on the 1x1 c3 shapes at the current code
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CASES="l3c1:--x3 l2c1:--x3 l4c1:--x3 l1c1:--x3 l3c3:--x3d,--dense l3c3:--x3p l2c3:--x3d,--dense l2c3:--x3p"
S="python tools/stamps.py"
cmd=""
for lib in s0 x3phs; do for c in l3c1:--x3 l2c1:--x3; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
B="python bench.py --no-cpu-baseline"
tools/gpu_steps.sh \
  "300|par10|CAPMI_LIB=ab/x3ph.so $T tests/test_gpu_x3.py tests/test_gpu_sk_handoff.py -k 'x3_dense or x3_conv or encoder_x3_matches or beta or handoff'" \
  "600|ab10|python tools/ab_inproc.py --libs base,ab/x3ph.so --cases '$CASES' --reps 20 --rounds 5" \
  "300|stamps10|${cmd% &&}" \
  "200|b10_base1|$B > gpurun_out/b10_base1.json" \
  "200|b10_x1|CAPMI_LIB=ab/x3ph.so $B > gpurun_out/b10_x1.json" \
  "200|b10_base2|$B > gpurun_out/b10_base2.json" \
  "200|b10_x2|CAPMI_LIB=ab/x3ph.so $B > gpurun_out/b10_x2.json"
