#!/bin/bash
# decoder-path A/B on one box: CAPMI_DEC_FUSED 0 / 1 / 2, sequential (enc + dec chains) and pipelined
for m in 0 1 2 0 1; do
  tools/gpu_steps.sh "200|ab_seq_$m|CAPMI_DEC_FUSED=$m python bench.py --no-cpu-baseline --no-roofline --sequential" || exit 1
done
for m in 0 1 0 1; do
  tools/gpu_steps.sh "200|ab_pipe_$m|CAPMI_DEC_FUSED=$m python bench.py --no-cpu-baseline --no-roofline" || exit 1
done
