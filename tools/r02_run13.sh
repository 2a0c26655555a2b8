#!/bin/bash
# fused dgrad weight pack (x3d B operand): bit-identity test, fine-tune parity, then the A/B
B="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
tools/gpu_steps.sh "400|t14|timeout -k 10 360 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|p_on|$B" "100|p_off|CAPMI_FT_PACK_X3=0 $B" "100|p_on2|$B" "100|p_off2|CAPMI_FT_PACK_X3=0 $B"
for f in gpurun_out/p_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
