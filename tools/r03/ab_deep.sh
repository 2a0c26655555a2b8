#!/bin/bash
# x3d two-deep A pipeline A/B: correctness (x3d / encoder x3 tests) then per-shape times, both builds
tools/gpu_steps.sh \
  "300|t_x3d|python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread -k 'x3d or encoder_x3_matches'" \
  "300|ab_deep|python -u tools/r03/conv_ab.py" \
  "300|ab_nodeep|CAPMI_LIB=ab/libcapmi_nodeep.so python -u tools/r03/conv_ab.py"
