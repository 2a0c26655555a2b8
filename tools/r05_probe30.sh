#!/bin/bash
# round 5, probe 30: the batched weight preparation (grid rows sized by the largest job, 32-bit index math, 1x1 and 3x3-dgrad jobs through LDS tiles): its tests, the
# fine-tune tests, config 4 with it and with the per-conv path (CAPMI_FT_WPREP_BATCH=0), alternating, and a trace
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python bench.py --config glove_finetune --steps 20 --warmup 3 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "600|ft_tests|$T tests/test_gpu_finetune.py" || exit $?
grep -q " passed" gpurun_out/ft_tests.log && ! grep -q " failed" gpurun_out/ft_tests.log || exit 1
tools/gpu_steps.sh "200|w1|$B" "200|w0|CAPMI_FT_WPREP_BATCH=0 $B" "200|w1b|$B" "200|w0b|CAPMI_FT_WPREP_BATCH=0 $B" \
  "300|wtr|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wtr -o t -- python $GRAFT_REPO_ROOT/bench.py --config glove_finetune --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > /dev/null && cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/wtr/t_results.db --top 60 > gpurun_out/wtr.md && rm -rf gpurun_out/wtr"
for f in w1 w0 w1b w0b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep weight_x3 gpurun_out/wtr.md | cut -c1-150
