#!/bin/bash
# x3 tile keep mask (CAPMI_X3_KEEP_TILE) on the fine-tune config: parity with all kept, then the A/B
B="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
tools/gpu_steps.sh "300|t13|CAPMI_X3_KEEP_TILE=3 timeout -k 10 280 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 250 --timeout-method thread" && \
tools/gpu_steps.sh "100|k0|$B" "100|k1|CAPMI_X3_KEEP_TILE=1 $B" "100|k2|CAPMI_X3_KEEP_TILE=2 $B" "100|k3|CAPMI_X3_KEEP_TILE=3 $B" \
  "100|k0b|$B" "100|k1b|CAPMI_X3_KEEP_TILE=1 $B" "100|k2b|CAPMI_X3_KEEP_TILE=2 $B" "100|k3b|CAPMI_X3_KEEP_TILE=3 $B"
for f in gpurun_out/k*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
