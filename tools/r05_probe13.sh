#!/bin/bash
# round 5, probe 13: interference knobs at the current code: stream-K worker count, stream priorities,
# data-parallel families
B="python bench.py --no-cpu-baseline --no-roofline"
steps=()
for r in 1 2; do
  for a in "base:" "sk240:CAPMI_SK_CUS=240" "sk224:CAPMI_SK_CUS=224" "swap:CAPMI_PIPE_PRIO=swap" "eq:CAPMI_PIPE_PRIO=equal" "fam5:CAPMI_SK_FAMILY_OFF=5"; do
    n=${a%%:*}; e=${a#*:}
    steps+=("200|b13_${n}_$r|$e $B > gpurun_out/b13_${n}_$r.json")
  done
done
tools/gpu_steps.sh "${steps[@]}"
