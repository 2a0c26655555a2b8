#!/bin/bash
# x3s + store-only epilogue: x3 kernel tests (incl. the encoder-level x3 tests), per-conv A/B table, bench line
tools/gpu_steps.sh \
  "400|t_x3|python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 200 --timeout-method thread -k 'not oversize'" \
  "300|conv_ab|python -u tools/r03/conv_ab.py" \
  "300|bench|python bench.py --no-cpu-baseline"
