#!/bin/bash
# round 4: beta epilogues with the C loads batched ahead of the stores -- parity (fine-tune, x3, decoder, GEMM
# suites), then the fine-tune and headline bench
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "600|t|$P tests/test_gpu_finetune.py tests/test_gpu_x3.py tests/test_gpu_gemm.py tests/test_gpu_decoder.py tests/test_gpu_split_gemm.py" \
 "200|f1|$B --config glove_finetune > gpurun_out/b18_f1.json" \
 "200|f2|$B --config glove_finetune > gpurun_out/b18_f2.json" \
 "150|h1|$B > gpurun_out/b18_h1.json"
