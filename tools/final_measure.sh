#!/bin/bash
# Closing measurement set for one config ($CFG): the default bench line, a rocprofv3 kernel trace of the same
# command, and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs); the databases are summarised on the box
# (gpurun_out/prof_$CFG.md, gpurun_out/pmc_traffic_$CFG.json) and removed (gpurun copies back <= 64 MiB)
R=$GRAFT_REPO_ROOT
CFG=${CFG:-attention}
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python $R/bench.py --config $CFG"
O=$R/gpurun_out
tools/gpu_steps.sh \
  "400|bench_$CFG|$B > $O/bench_$CFG.json" \
  "400|prof_$CFG|$P --kernel-trace --stats -d $O/prof_$CFG -o bench -- $B --no-cpu-baseline" \
  "300|pmcf_$CFG|$P --pmc FETCH_SIZE -d $O/pmcf_$CFG -o pmc -- $B --no-cpu-baseline --steps 2 --warmup 1 --no-roofline" \
  "300|pmcw_$CFG|$P --pmc WRITE_SIZE -d $O/pmcw_$CFG -o pmc -- $B --no-cpu-baseline --steps 2 --warmup 1 --no-roofline" || exit $?
python tools/prof_summary.py $O/prof_$CFG/bench_results.db --top 45 > $O/prof_$CFG.md && \
python tools/pmc_traffic.py $O/pmcf_$CFG/pmc_results.db $O/pmcw_$CFG/pmc_results.db \
  --command "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- python bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 1 --no-roofline" \
  > $O/pmc_traffic_$CFG.json && rm -rf $O/prof_$CFG $O/pmcf_$CFG $O/pmcw_$CFG
