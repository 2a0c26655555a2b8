#!/bin/bash
# Round-1 measurement set on one MI355X: GPU tests, the three bench configs (JSON lines), kernel-trace
# profiles of the headline and the bf16 config, PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs)
# for the traffic figures, in four calls (a: tests+benches+trace, b: bf16 trace, c/d: PMC) so that
# each call's gpurun_out stays under 64 MiB. Each step under its own time limit; stops at the first fault/timeout.
R=$GRAFT_REPO_ROOT
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
case "$1" in
a) tools/gpu_steps.sh \
  "400|tests|python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread" \
  "300|bench|python bench.py --steps 20 --warmup 3" \
  "300|bertbench|python bench.py --config bert_attention --steps 20 --warmup 3" \
  "300|ftbench|python bench.py --config glove_finetune --steps 10 --warmup 2" \
  "300|prof|$P --kernel-trace --stats -d $R/gpurun_out/prof_final -o bench -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline" ;;
b) tools/gpu_steps.sh \
  "300|profbert|$P --kernel-trace --stats -d $R/gpurun_out/prof_bert -o bench -- python $R/bench.py --config bert_attention --steps 10 --warmup 3 --no-cpu-baseline" ;;
c) tools/gpu_steps.sh \
  "300|pmcf|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o pmc -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "300|pmcw|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o pmc -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" ;;
d) tools/gpu_steps.sh \
  "300|pmcfb|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_bert -o pmc -- python $R/bench.py --config bert_attention --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "300|pmcwb|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_bert -o pmc -- python $R/bench.py --config bert_attention --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" ;;
e) tools/gpu_steps.sh \
  "300|pmcfb|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_bert -o pmc -- python $R/bench.py --config bert_attention --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "300|pmcwb|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_bert -o pmc -- python $R/bench.py --config bert_attention --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "300|pmcff|$P --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_ft -o pmc -- python $R/bench.py --config glove_finetune --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" \
  "300|pmcwf|$P --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_ft -o pmc -- python $R/bench.py --config glove_finetune --steps 2 --warmup 1 --no-cpu-baseline --no-roofline" ;;
esac
