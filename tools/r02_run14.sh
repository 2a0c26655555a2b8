#!/bin/bash
# 1x1 fine-tune dgrads on the weight as k rows (no per-step pack): parity, then the A/B
B="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
tools/gpu_steps.sh "400|t15|timeout -k 10 360 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 300 --timeout-method thread -k 'matches_oracle'" && \
tools/gpu_steps.sh "100|q_on|CAPMI_FT_DGRAD1_KROWS=1 $B" "100|q_off|$B" "100|q_on2|CAPMI_FT_DGRAD1_KROWS=1 $B" "100|q_off2|$B"
for f in gpurun_out/q_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
