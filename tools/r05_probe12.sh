#!/bin/bash
# round 5, probe 12: the fused decoder recurrence (CAPMI_DEC_FUSED 1 / 2, decoder_step.hip) at the current code
B="python bench.py --no-cpu-baseline --no-roofline"
steps=()
for r in 1 2; do
  for a in "base:" "f1:CAPMI_DEC_FUSED=1" "f2:CAPMI_DEC_FUSED=2"; do
    n=${a%%:*}; e=${a#*:}
    steps+=("200|b12_${n}_$r|$e $B > gpurun_out/b12_${n}_$r.json")
  done
done
for a in "base:" "f1:CAPMI_DEC_FUSED=1" "f2:CAPMI_DEC_FUSED=2"; do
  n=${a%%:*}; e=${a#*:}
  steps+=("300|pp12_$n|$e python tools/pipe_parts.py --steps 30 > gpurun_out/pp12_$n.txt")
done
tools/gpu_steps.sh "${steps[@]}"
