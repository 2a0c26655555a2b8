#!/bin/bash
# round 4: x3w tests (operands held), the wide x3d probe, x3w timing, the decoder flip rule at B = 64
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -s"
tools/gpu_steps.sh \
 "300|x3w|$P tests/test_gpu_finetune.py -k x3w" \
 "200|wide|python -u tools/r04/wide_probe.py > gpurun_out/wide_probe.txt" \
 "200|x3wt|python -u tools/r04/x3w_debug.py > gpurun_out/x3w_debug.txt" \
 "600|flips|python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -s tests/test_gpu_headline_parity.py tests/test_gpu_bench_paths.py" \
 "120|bench|python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b4_a.json"
