#!/bin/bash
# fine-tune config after the x3d dgrads: parity (all dgrad routes), bench line, kernel trace, PMC passes
R=$GRAFT_REPO_ROOT
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python $R/bench.py --config glove_finetune --no-cpu-baseline"
tools/gpu_steps.sh "400|t12|timeout -k 10 360 python -u -m pytest tests/test_gpu_finetune.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "150|bench_ft|python bench.py --config glove_finetune --no-cpu-baseline" \
  "300|prof_ft|$P --kernel-trace --stats -d $R/gpurun_out/prof_ft -o bench -- $B --steps 10 --warmup 3 --no-roofline" \
  "300|pmcf_ft|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_ft -o pmc -- $B --steps 1 --warmup 1 --no-roofline" \
  "300|pmcw_ft|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_ft -o pmc -- $B --steps 1 --warmup 1 --no-roofline"
