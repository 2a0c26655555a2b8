#!/bin/bash
# round 5, probe 1: per-conv times of the 1x1 / 3x3 x3 kernels (base, LATEBAR, PRIO builds), the in-kernel phase
# stamps of the same launches, and stream-K vs data-parallel x3d on layer3 c3
G="python tools/gemm_one.py --reps 30"
S="python tools/stamps.py"
CASES="l3c3:--x3d,--dense l2c3:--x3d,--dense l4c3:--x3d,--dense l3c1:--x3 l2c1:--x3 l3c2:--x3p l2c2:--x3p l3c2s:--x3d l4c2:--x3d"
steps=()
for lib in base latebar prio; do
  L=""; [ $lib != base ] && L="CAPMI_LIB=ab/$lib.so"
  cmd=""
  for c in $CASES; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd $L $G --shape $sh ${f//,/ } &&"; done
  steps+=("240|t_$lib|${cmd% &&}")
done
cmd=""
for c in $CASES; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/stamp.so $S --shape $sh ${f//,/ } &&"; done
steps+=("240|stamps|${cmd% &&}")
steps+=("120|t_dp|CAPMI_SK_FAMILY_OFF=5 $G --shape l3c3 --x3d --dense && CAPMI_SK_FAMILY_OFF=5 CAPMI_LIB=ab/stamp.so $S --shape l3c3 --x3d --dense && CAPMI_SK_FAMILY_OFF=0 $G --shape l3c1 --x3 && CAPMI_SK_FAMILY_OFF=7 $G --shape l3c2 --x3p")
tools/gpu_steps.sh "${steps[@]}"
