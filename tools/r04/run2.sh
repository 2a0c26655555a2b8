#!/bin/bash
# round 4: x3w and fused-tail tests, the wide x3d probe, x3w timing, the decoder flip rule at B = 64, tail A/B
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "300|x3w|$P tests/test_gpu_finetune.py -k x3w" \
 "300|tail|$P tests/test_gpu_x3.py -k tail" \
 "200|wide|python -u tools/r04/wide_probe.py > gpurun_out/wide_probe.txt" \
 "200|x3wt|python -u tools/r04/x3w_debug.py > gpurun_out/x3w_debug.txt" \
 "120|b_tail|$B > gpurun_out/b4_tail.json" \
 "120|b_notail|CAPMI_X3_TAIL=0 $B > gpurun_out/b4_notail.json" \
 "120|b_tail2|$B > gpurun_out/b4_tail2.json" \
 "120|b_notail2|CAPMI_X3_TAIL=0 $B > gpurun_out/b4_notail2.json" \
 "600|flips|python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -s tests/test_gpu_headline_parity.py tests/test_gpu_bench_paths.py"
