#!/bin/bash
# split-staged decoder GEMMs: kernel tests, decoder parity, then the bench A/B (x3 / fp32 / bf16 decoder GEMMs)
tools/gpu_steps.sh "400|split|python -u -m pytest tests/test_gpu_split_gemm.py -x -q --timeout 120 --timeout-method thread" && \
tools/gpu_steps.sh "500|decpar|python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "200|b_att_x3|python bench.py --no-cpu-baseline" "200|b_att_fp32|python bench.py --no-cpu-baseline --no-roofline --dec fp32" \
  "200|b_bert_bf16|python bench.py --config bert_attention --no-cpu-baseline" "200|b_bert_fp32dec|python bench.py --config bert_attention --no-cpu-baseline --no-roofline --dec fp32"
