#!/bin/bash
# x3d dense-rows prologue: x3 tests, per-conv table, bench pair (old form: CAPMI_X3D_CONV1X1=1 is not a switch;
# the comparison is the conv table's x3d column against profiles/r03_conv_ab_x3s.md)
tools/gpu_steps.sh \
  "400|t_x3|python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_bench_paths.py -x -q --timeout 300 --timeout-method thread -k 'not oversize'" \
  "300|conv_ab|python -u tools/r03/conv_ab.py" \
  "300|hl|python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_noplain|CAPMI_X3_PLAIN_EPI=0 python bench.py --no-cpu-baseline --no-roofline" \
  "300|ft|python bench.py --config glove_finetune --no-cpu-baseline --no-roofline" \
  "300|ft_old|CAPMI_X3_PLAIN_EPI=0 CAPMI_FT_DGRAD1_X3D=0 python bench.py --config glove_finetune --no-cpu-baseline --no-roofline"
