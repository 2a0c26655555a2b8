#!/bin/bash
# bf16 store-only epilogue: bf16 GEMM / encoder tests, config-5 bench pair on one box
tools/gpu_steps.sh \
  "400|t_bf16|python -u -m pytest tests/test_gpu_bf16io.py tests/test_gpu_bf16.py tests/test_gpu_bert.py tests/test_gpu_bench_paths.py -x -q --timeout 300 --timeout-method thread" \
  "300|bf_new|python bench.py --config bert_attention --no-cpu-baseline --no-roofline" \
  "300|bf_old|CAPMI_X3_PLAIN_EPI=0 python bench.py --config bert_attention --no-cpu-baseline --no-roofline" \
  "300|bf_new2|python bench.py --config bert_attention --no-cpu-baseline --no-roofline" \
  "300|bf_old2|CAPMI_X3_PLAIN_EPI=0 python bench.py --config bert_attention --no-cpu-baseline --no-roofline"
