#!/bin/bash
# round 5, probe 28: the fine-tune step's deferred weight-gradient sums (CAPMI_GEMM_X3W_DEFER + one
# capmi_splitk_reduce_batch): the fine-tune tests, then config 4 with it (default) and without
# (CAPMI_FT_WGRAD_DEFER=0), alternating
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python bench.py --config glove_finetune --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "600|ft_tests|$T tests/test_gpu_finetune.py tests/test_gpu_bench_paths.py" || exit $?
grep -q " passed" gpurun_out/ft_tests.log && ! grep -q " failed" gpurun_out/ft_tests.log || exit 1
tools/gpu_steps.sh "200|d1|$B" "200|d0|CAPMI_FT_WGRAD_DEFER=0 $B" "200|d1b|$B" "200|d0b|CAPMI_FT_WGRAD_DEFER=0 $B"
for f in d1 d0 d1b d0b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
