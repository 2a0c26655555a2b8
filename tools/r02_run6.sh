#!/bin/bash
# x3 transposed staging (conflict-free k-pair store, 64x64 tiles): decoder x3 vs fp32 in the headline,
# fine-tune x3 wgrads / decoder; tests first
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "400|t6|python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_finetune.py tests/test_gpu_decoder.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|h_x3|$B --dec x3" "100|h_fp32|$B --dec fp32" "100|h_x3b|$B --dec x3" "100|h_fp32b|$B --dec fp32" \
  "100|f_x3|$B --config glove_finetune --dec x3" "100|f_fp32|$B --config glove_finetune --dec fp32" \
  "100|f_x3_nowg|CAPMI_FT_WGRAD_X3=0 $B --config glove_finetune --dec x3" "100|f_x3b|$B --config glove_finetune --dec x3"
for f in gpurun_out/h_*.log gpurun_out/f_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
