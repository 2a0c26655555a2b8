#!/bin/bash
# fused bottleneck tails: kernel + encoder bit-identity tests, the encoder-level x3 tests, bench both arms
tools/gpu_steps.sh \
  "400|t_x3|python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 200 --timeout-method thread -k 'not oversize'" \
  "300|bench_tail|python bench.py --no-cpu-baseline" \
  "300|bench_notail|CAPMI_X3_TAIL=0 python bench.py --no-cpu-baseline --no-roofline"
