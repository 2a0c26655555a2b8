#!/bin/bash
# kernel trace of the fine-tune config at HEAD
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh "300|prof_ft2|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ft2 -o bench -- python $R/bench.py --config glove_finetune --no-cpu-baseline --steps 10 --warmup 3 --no-roofline"
