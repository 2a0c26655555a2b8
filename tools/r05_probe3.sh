#!/bin/bash
# round 5, probe 3: x3p + x3d with the mid-tile barrier and the staging behind it (X3P_PHASE): parity of every
# x3p / x3d path on the variant, same-process A/B of the builds per conv shape, phase stamps
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
CASES="l3c2:--x3p l2c2:--x3p l3c3:--x3d,--dense l2c3:--x3d,--dense l4c3:--x3d,--dense l4c2:--x3d l3c2s:--x3d ds3:--x3d l4c1:--x3d,--nopro l2c2s:--x3d"
S="python tools/stamps.py"
cmd=""
for lib in stamp ph2s; do for c in l3c2:--x3p l3c3:--x3d,--dense l4c2:--x3d; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
tools/gpu_steps.sh \
  "300|par3|CAPMI_LIB=ab/ph2.so $T tests/test_gpu_x3.py -k 'x3p or x3d or encoder_x3_matches'" \
  "600|ab3|python tools/ab_inproc.py --libs base,ab/ph1.so,ab/ph2.so,ab/ph3.so,ab/ph2v2.so --cases '$CASES' --reps 20 --rounds 5" \
  "300|stamps3|${cmd% &&}"
