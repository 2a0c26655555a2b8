#!/bin/bash
# layer1 3x3 on x3p 256x64 (BK 32): x3p / encoder x3 tests, per-conv layer1 table, bench pairs
tools/gpu_steps.sh \
  "400|t_x3p|python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_bench_paths.py -x -q --timeout 300 --timeout-method thread -k 'x3p or encoder_x3 or bench_path or b64'" \
  "200|ab_l1|python -u tools/r03/conv_ab.py --only l1" \
  "300|hl_new|python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_old|CAPMI_X3P64=0 python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_new2|python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_old2|CAPMI_X3P64=0 python bench.py --no-cpu-baseline --no-roofline"
