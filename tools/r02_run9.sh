#!/bin/bash
# fine-tune 3x3 / sub-pixel dgrads on x3d: fine-tune parity (x3 + fp32 + bf16), then the A/B
B="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
tools/gpu_steps.sh "400|t10|timeout -k 10 360 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|g_on|$B" "100|g_off|CAPMI_FT_DGRAD_X3D=0 $B" "100|g_on2|$B" "100|g_off2|CAPMI_FT_DGRAD_X3D=0 $B"
for f in gpurun_out/g_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
