#!/bin/bash
# round 5, probe 9: what the x3d A split costs (timing-only X3D_NOSPLIT build), the hand-off stress test
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CASES="l3c3:--x3d,--dense l2c3:--x3d,--dense l4c3:--x3d,--dense l4c2:--x3d l3c2s:--x3d ds3:--x3d l4c1:--x3d,--nopro"
S="python tools/stamps.py"
cmd=""
for lib in s0 nosplits; do for c in l3c3:--x3d,--dense ds3:--x3d; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
tools/gpu_steps.sh \
  "400|par9|$T tests/test_gpu_sk_handoff.py" \
  "600|ab9|python tools/ab_inproc.py --libs base,ab/nosplit.so --cases '$CASES' --reps 20 --rounds 5" \
  "300|stamps9|${cmd% &&}"
