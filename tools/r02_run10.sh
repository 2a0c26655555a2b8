#!/bin/bash
# fine-tune 1x1 dgrads on x3d too: fine-tune parity, then the A/B
B="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
tools/gpu_steps.sh "400|t11|timeout -k 10 360 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|h_on|$B" "100|h_off|CAPMI_FT_DGRAD1_X3D=0 $B" "100|h_on2|$B" "100|h_off2|CAPMI_FT_DGRAD1_X3D=0 $B"
for f in gpurun_out/h_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
