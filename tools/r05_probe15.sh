#!/bin/bash
# round 5, probe 15: what bounds x3p's phase loop (timing-only builds with stamps: no DMA, no LDS reads, neither,
# zero-size descriptors) on layer3 / layer2 3x3
S="python tools/stamps.py"
cmd=""
for lib in s0 s1 s2 s3 pr; do for c in l3c2:--x3p l2c2:--x3p; do sh=${c%%:*}; f=${c#*:}; cmd="$cmd CAPMI_LIB=ab/$lib.so $S --shape $sh ${f//,/ } &&"; done; done
tools/gpu_steps.sh "400|stamps15|${cmd% &&}"
