#!/bin/bash
# kernel trace of the pipelined bench (csv, for tools/timeline.py) -> gpurun_out/tl_$1/
R=$GRAFT_REPO_ROOT
N=${1:-pipe}; shift
tools/gpu_steps.sh "300|tl_$N|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_$N -o tl -- python $R/bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3 $*"
