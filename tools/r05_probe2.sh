#!/bin/bash
# round 5, probe 2: x3p with the DMA issued after the mid-tile barrier (X3P_PHASE 1-3): parity (x3p tests and
# the encoder on the variant library), per-conv times, phase stamps
G="python tools/gemm_one.py --reps 30"
S="python tools/stamps.py"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
CASES="l3c2:--x3p l2c2:--x3p l3c3:--x3p l3c3:--x3d,--dense l3c1:--x3"
steps=("300|par_ph2|CAPMI_LIB=ab/ph2.so $T tests/test_gpu_x3.py -k 'x3p or encoder_x3_matches'")
for lib in base ph1 ph2 ph3 base; do
  L=""; [ $lib != base ] && L="CAPMI_LIB=ab/$lib.so"
  cmd=""
  for c in $CASES; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd $L $G --shape $sh ${f//,/ } &&"; done
  steps+=("240|t2_$lib|${cmd% &&}")
done
cmd=""
for lib in stamp ph2s; do for c in $CASES; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
steps+=("300|stamps2|${cmd% &&}")
tools/gpu_steps.sh "${steps[@]}"
