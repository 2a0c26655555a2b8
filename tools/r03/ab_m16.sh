#!/bin/bash
# x3p/x3d MFMA shape A/B (16x16x32 default vs 32x32x16): correctness of the x3p / x3d kernels and the
# encoder, then per-shape times of both builds
tools/gpu_steps.sh \
  "300|t_x3|python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread -k 'not oversize'" \
  "300|ab_m16|python -u tools/r03/conv_ab.py" \
  "300|ab_m32|CAPMI_LIB=ab/libcapmi_m32.so python -u tools/r03/conv_ab.py"
