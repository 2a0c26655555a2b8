#!/bin/bash
# Round-1 measurement set on one MI355X: GPU tests, bench (JSON line), kernel-trace profile of
# the same bench command, two PMC passes (FETCH_SIZE, WRITE_SIZE) for the traffic figure.
# Each step under its own time limit; stops at the first fault/abort/timeout.
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
  "400|tests|python -m pytest tests -m gpu -q -x" \
  "300|bench|python bench.py --steps 20 --warmup 3" \
  "400|prof|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o bench -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline" \
  "400|pmcf|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o pmc -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "400|pmcw|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o pmc -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline"
