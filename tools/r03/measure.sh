#!/bin/bash
# Round-3 measurement set on one MI355X (each step under its own limit; stops at the first fault):
#   b: the default bench line -> gpurun_out/bench_$TAG.json
#   t: rocprofv3 kernel trace of the same bench command -> gpurun_out/prof_$TAG/
R=$GRAFT_REPO_ROOT
TAG=${TAG:-base}
CFG=${CFG:-attention}
EXTRA=${EXTRA:-}
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python $R/bench.py --config $CFG $EXTRA"
tools/gpu_steps.sh \
  "400|bench_$TAG|$B > $R/gpurun_out/bench_$TAG.json" \
  "400|prof_$TAG|$P --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o bench -- $B --no-cpu-baseline"
