#!/bin/bash
# bf16 encoder with the BN prologue folded into the GEMM: bit-identity + bf16 tests, bench arms (0 / 2 / 3)
tools/gpu_steps.sh \
  "400|t_bf16|python -u -m pytest tests/test_gpu_bf16io.py tests/test_gpu_bf16.py -x -v --timeout 200 --timeout-method thread" \
  "300|bench_bf_fold2|python bench.py --config bert_attention --no-cpu-baseline" \
  "300|bench_bf_fold0|CAPMI_BF16_FOLD=0 python bench.py --config bert_attention --no-cpu-baseline --no-roofline" \
  "300|bench_bf_fold3|CAPMI_BF16_FOLD=3 python bench.py --config bert_attention --no-cpu-baseline --no-roofline"
