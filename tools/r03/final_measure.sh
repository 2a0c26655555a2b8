#!/bin/bash
# Round-3 measurement set for one config ($CFG): the default bench line, a rocprofv3 kernel trace of the same
# command, and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) -> gpurun_out/{bench,prof,pmcf,pmcw}_$CFG
R=$GRAFT_REPO_ROOT
CFG=${CFG:-attention}
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python $R/bench.py --config $CFG"
tools/gpu_steps.sh \
  "400|bench_$CFG|$B > $R/gpurun_out/bench_$CFG.json" \
  "400|prof_$CFG|$P --kernel-trace --stats -d $R/gpurun_out/prof_$CFG -o bench -- $B --no-cpu-baseline" \
  "300|pmcf_$CFG|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_$CFG -o pmc -- $B --no-cpu-baseline --steps 2 --warmup 1 --no-roofline" \
  "300|pmcw_$CFG|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_$CFG -o pmc -- $B --no-cpu-baseline --steps 2 --warmup 1 --no-roofline"
