#!/bin/bash
# elementwise kernels: oversize x3 route test, then a kernel trace of the bench (per-shape durations)
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
  "300|t_over|python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread -k 'oversize'" \
  "400|prof_elt|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_elt -o bench -- python $R/bench.py --no-cpu-baseline"
