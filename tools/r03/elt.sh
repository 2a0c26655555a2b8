#!/bin/bash
# channel-stationary elementwise kernels: their tests, the encoder x3 tests, bench
tools/gpu_steps.sh \
  "400|t_elt|python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_x3.py tests/test_gpu_bn_fused.py -x -q --timeout 200 --timeout-method thread -k 'bn_add_relu or split3 or encoder_x3 or bn_fused or fused_tail'" \
  "300|bench|python bench.py --no-cpu-baseline"
