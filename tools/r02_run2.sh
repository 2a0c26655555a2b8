#!/bin/bash
# RCCL one-rank DP tests, a forced-RCCL bench line, and kernel traces of the sequential step (decoder
# and encoder chains alone) and the pipelined step, for tools/timeline.py
R=$GRAFT_REPO_ROOT
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
tools/gpu_steps.sh \
  "300|rccl_test|python -u -m pytest tests/test_gpu_dp.py -k rccl -x -v --timeout 200 --timeout-method thread" \
  "200|bench_rccl|CAPMI_DIST_FORCE=1 python bench.py --no-cpu-baseline" \
  "200|bench_seq|python bench.py --no-cpu-baseline --sequential --no-roofline" \
  "300|tl_seq|$P --kernel-trace --output-format csv -d $R/gpurun_out/tl_seq -o tl -- python $R/bench.py --no-cpu-baseline --sequential --no-roofline --steps 10 --warmup 3" \
  "300|tl_pipe|$P --kernel-trace --output-format csv -d $R/gpurun_out/tl_pipe -o tl -- python $R/bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
