#!/bin/bash
# round 4: x3c with the weight ring and slice prefetch (parity first), its time, bench A/B, then the full GPU
# suite and smoke
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "200|x3c|$P tests/test_gpu_x3.py -k x3c" \
 "200|x3c_t|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/x3c_time2.txt" \
 "120|b_d|$B > gpurun_out/b9_d.json" \
 "120|b_c0|CAPMI_X3C=0 $B > gpurun_out/b9_c0.json" \
 "120|b_d2|$B > gpurun_out/b9_d2.json" \
 "120|b_c02|CAPMI_X3C=0 $B > gpurun_out/b9_c02.json" \
 "900|suite|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200|smoke|python -c 'import __graft_entry__ as g; g.smoke()'"
