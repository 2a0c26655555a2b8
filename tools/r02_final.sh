#!/bin/bash
# round-2 closing measurement: full GPU suite, the default bench line (with the CPU baseline), the
# other configs' lines, and a kernel trace of the headline
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh "700|gpu_all|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "300|bench_default|python bench.py" \
  "150|bench_ft|python bench.py --config glove_finetune --no-cpu-baseline" \
  "150|bench_bert|python bench.py --config bert_attention --no-cpu-baseline" \
  "300|prof_att|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o bench -- python $R/bench.py --no-cpu-baseline --steps 10 --warmup 3"
