#!/bin/bash
# x3d routing: encoder-level parity (x3 encoder, fine-tune, whole step), then the A/B
B="python bench.py --no-cpu-baseline --no-roofline"
export CAPMI_X3D=1
tools/gpu_steps.sh "500|t9|timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_finetune.py tests/test_gpu_train_step.py tests/test_gpu_headline_parity.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|d_on|$B" "100|d_off|CAPMI_X3D=0 $B" "100|d_on2|$B" "100|d_off2|CAPMI_X3D=0 $B" \
  "100|d_ft_on|$B --config glove_finetune" "100|d_ft_off|CAPMI_X3D=0 $B --config glove_finetune"
for f in gpurun_out/d_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
