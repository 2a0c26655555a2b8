#!/bin/bash
# x3p with 256 x 64 tiles (layer1's 3x3): x3p tests, per-conv A/B (layer1)
tools/gpu_steps.sh \
  "400|t_x3p|python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 200 --timeout-method thread -k 'x3p or x3d or encoder_x3_matches'" \
  "300|conv_ab_l1|python -u tools/r03/conv_ab.py --only l1" \
  "300|conv_ab_l1_bk32|CAPMI_X3P_BK=32 python -u tools/r03/conv_ab.py --only l1 --arms x3p"
