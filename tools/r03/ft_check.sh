#!/bin/bash
# fine-tune: tests (encoder backward, the whole step, x3 kernels), bench with the beta epilogue and 1x1 dgrads on x3d
tools/gpu_steps.sh \
  "600|t_ft|python -u -m pytest tests/test_gpu_finetune.py tests/test_gpu_x3.py tests/test_gpu_bench_paths.py -x -q --timeout 300 --timeout-method thread" \
  "300|ft_new|python bench.py --config glove_finetune --no-cpu-baseline --no-roofline" \
  "300|ft_old|CAPMI_X3_PLAIN_EPI=0 CAPMI_FT_DGRAD1_X3D=0 python bench.py --config glove_finetune --no-cpu-baseline --no-roofline" \
  "300|ft_new2|python bench.py --config glove_finetune --no-cpu-baseline --no-roofline"
