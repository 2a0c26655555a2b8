#!/bin/bash
# round 5, probe 7: transposed 16x16 accumulators + 16-B epilogue stores (X3P_TEPI): parity, same-process A/B,
# stamps, SQ passes on the bench's instantiations, a bench pair
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
CASES="l3c2:--x3p l2c2:--x3p l3c3:--x3d,--dense l2c3:--x3d,--dense l4c3:--x3d,--dense l4c2:--x3d l3c2s:--x3d ds3:--x3d l4c1:--x3d,--nopro l2c2s:--x3d"
S="python tools/stamps.py"
cmd=""
for lib in s0 ts; do for c in l3c3:--x3d,--dense l2c3:--x3d,--dense l3c2:--x3p; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
B="python bench.py --no-cpu-baseline"
tools/gpu_steps.sh \
  "300|par7|CAPMI_LIB=ab/t.so $T tests/test_gpu_x3.py -k 'x3p or x3d or encoder_x3_matches or beta'" \
  "600|ab7|python tools/ab_inproc.py --libs base,ab/t.so --cases '$CASES' --reps 20 --rounds 5" \
  "300|stamps7|${cmd% &&}" \
  "200|b7_base1|$B > gpurun_out/b7_base1.json" \
  "200|b7_t1|CAPMI_LIB=ab/t.so $B > gpurun_out/b7_t1.json" \
  "200|b7_base2|$B > gpurun_out/b7_base2.json" \
  "200|b7_t2|CAPMI_LIB=ab/t.so $B > gpurun_out/b7_t2.json" \
  "600|sq7|CASES='l3c3:--x3d,--dense l3c3:--x3p l3c2:--x3p l3c1:--x3 l2c3:--x3d,--dense' bash tools/sq.sh"
