#!/bin/bash
# Round-2 measurement set on one MI355X (each step under its own limit; stops at the first fault):
#   t: kernel-trace profile of the bench (config $CFG, default attention) -> gpurun_out/prof_<cfg>/
#   f/w: FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) -> gpurun_out/pmc_{fetch,write}_<cfg>/
R=$GRAFT_REPO_ROOT
CFG=${CFG:-attention}
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python $R/bench.py --config $CFG --no-cpu-baseline"
tools/gpu_steps.sh \
  "300|prof_$CFG|$P --kernel-trace --stats -d $R/gpurun_out/prof_$CFG -o bench -- $B --steps 10 --warmup 3" \
  "300|pmcf_$CFG|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$CFG -o pmc -- $B --steps 2 --warmup 1 --no-roofline" \
  "300|pmcw_$CFG|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$CFG -o pmc -- $B --steps 2 --warmup 1 --no-roofline"
