#!/bin/bash
# round 5, probe 11: decoder per-timestep GEMM workgroup targets (CAPMI_DEC_WGS) beside the encoder stream
B="python bench.py --no-cpu-baseline --no-roofline"
steps=()
for r in 1 2; do
  for a in "base:" "d128:CAPMI_DEC_WGS=128" "d64:CAPMI_DEC_WGS=64" "d32:CAPMI_DEC_WGS=32"; do
    n=${a%%:*}; e=${a#*:}
    steps+=("200|b11_${n}_$r|$e $B > gpurun_out/b11_${n}_$r.json")
  done
done
tools/gpu_steps.sh "${steps[@]}"
