#!/bin/bash
# round 4: x3c with the fixed band swizzle: parity, time, SQ, bench pair
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "200|x3c|$P tests/test_gpu_x3.py -k 'x3c or encoder_x3_matches'" \
 "200|x3c_t|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/x3c_time3.txt" \
 "120|b_d|$B > gpurun_out/b10_d.json" \
 "120|b_c0|CAPMI_X3C=0 $B > gpurun_out/b10_c0.json" \
 "300|sq|CASES='l1c2:x3c' bash tools/r03/sq.sh"
