#!/bin/bash
# gemm_nt store-only epilogue: decoder / split GEMM / fine-tune / train-step tests, headline + fine-tune bench pairs
tools/gpu_steps.sh \
  "700|t_nt|python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_split_gemm.py tests/test_gpu_decoder.py tests/test_gpu_finetune.py tests/test_gpu_train_step.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread" \
  "300|hl_new|python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_old|CAPMI_X3_PLAIN_EPI=0 python bench.py --no-cpu-baseline --no-roofline" \
  "300|hl_new2|python bench.py --no-cpu-baseline --no-roofline"
