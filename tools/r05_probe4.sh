#!/bin/bash
# round 5, probe 4: x3d with the split spread over the whole k-tile behind a block-3 barrier (X3D_V2) and x3p
# with the DMA behind a mid-tile barrier (X3P_PHASE=2): parity on the variant, same-process A/B per conv shape,
# phase stamps, two bench pairs
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
CASES="l3c2:--x3p l3c3:--x3d,--dense l2c3:--x3d,--dense l4c3:--x3d,--dense l4c2:--x3d l3c2s:--x3d ds3:--x3d l4c1:--x3d,--nopro l2c2s:--x3d"
S="python tools/stamps.py"
cmd=""
for lib in v2s; do for c in l3c3:--x3d,--dense l4c2:--x3d ds3:--x3d; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
  "300|par5|CAPMI_LIB=ab/v2.so $T tests/test_gpu_x3.py -k 'x3p or x3d or encoder_x3_matches'" \
  "600|ab5|python tools/ab_inproc.py --libs base,ab/p2.so,ab/v2.so,ab/v2b.so --cases '$CASES' --reps 20 --rounds 5" \
  "300|stamps5|${cmd% &&}" \
  "200|b5_p2_1|CAPMI_LIB=ab/p2.so $B > gpurun_out/b5_p2_1.json" \
  "200|b5_v2_1|CAPMI_LIB=ab/v2.so $B > gpurun_out/b5_v2_1.json" \
  "200|b5_p2_2|CAPMI_LIB=ab/p2.so $B > gpurun_out/b5_p2_2.json" \
  "200|b5_v2_2|CAPMI_LIB=ab/v2.so $B > gpurun_out/b5_v2_2.json"
