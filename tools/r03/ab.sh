#!/bin/bash
# Environment-switch A/B of the bench (DESIGN.md 4.9 lists the switches; 4.12 the arms measured and not taken).
# usage: CFG=attention ARMS="base: sk1:CAPMI_SK_FAMILY_OFF=0 bf16sk:CAPMI_BF16_SK=1" tools/r03/ab.sh
# Each arm "<name>:<VAR=value,VAR=value>" runs one bench line -> gpurun_out/ab_<name>.json, under its own limit.
CFG=${CFG:-attention}
steps=()
for arm in ${ARMS:-base:}; do
  name=${arm%%:*}; envs=${arm#*:}
  steps+=("300|ab_$name|${envs//,/ } python bench.py --config $CFG --no-cpu-baseline --no-roofline > gpurun_out/ab_$name.json")
done
tools/gpu_steps.sh "${steps[@]}"
