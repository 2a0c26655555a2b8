#!/bin/bash
# round 5, probe 27: the fine-tune step's batched weight preparation (capmi_weight_x3_batch): its tests and the
# fine-tune tests, then config 4 with it (default) and without (CAPMI_FT_WPREP_BATCH=0), alternating
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python bench.py --config glove_finetune --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "600|ft_tests|$T tests/test_gpu_finetune.py tests/test_gpu_bench_paths.py" || exit $?
grep -q " passed" gpurun_out/ft_tests.log && ! grep -q " failed" gpurun_out/ft_tests.log || exit 1
tools/gpu_steps.sh "200|w1|$B" "200|w0|CAPMI_FT_WPREP_BATCH=0 $B" "200|w1b|$B" "200|w0b|CAPMI_FT_WPREP_BATCH=0 $B"
for f in w1 w0 w1b w0b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
