#!/bin/bash
# round 5, probe 22: gemm_x3 stream-K again now that the hand-off is the sc1 form (CAPMI_SK_FAMILY_OFF=0 vs the
# default 1): the layer c1 shapes alone, x3d on them, then the headline step alternating
G="python tools/gemm_one.py --reps 50"
s=""
for sh in l3c1 l2c1 l4c1 l1c1; do
  s="$s CAPMI_SK_FAMILY_OFF=1 $G --shape $sh --x3 && CAPMI_SK_FAMILY_OFF=0 $G --shape $sh --x3 && $G --shape $sh --x3d --dense --nopro &&"
done
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "200|c1_alone|${s% &&}" \
  "200|b1|CAPMI_SK_FAMILY_OFF=1 $B" "200|b0|CAPMI_SK_FAMILY_OFF=0 $B" \
  "200|b1b|CAPMI_SK_FAMILY_OFF=1 $B" "200|b0b|CAPMI_SK_FAMILY_OFF=0 $B"
