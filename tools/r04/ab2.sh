#!/bin/bash
# round 4 A/B: stream-K hand-off ordering (release / acquire separately) and the x3d routing
B="python bench.py --no-cpu-baseline --no-roofline"
L=$PWD/ab
tools/gpu_steps.sh \
 "120|b_pk|CAPMI_LIB=$L/pk.so $B > gpurun_out/b2_pk.json" \
 "120|b_rel|CAPMI_LIB=$L/relonly.so $B > gpurun_out/b2_rel.json" \
 "120|b_acq|CAPMI_LIB=$L/acqonly.so $B > gpurun_out/b2_acq.json" \
 "120|b_mm|$B > gpurun_out/b2_mm.json" \
 "120|b_mm_noroute|CAPMI_R4_ROUTE=0 $B > gpurun_out/b2_mm_noroute.json" \
 "120|b_pk2|CAPMI_LIB=$L/pk.so $B > gpurun_out/b2_pk2.json" \
 "120|b_rel2|CAPMI_LIB=$L/relonly.so $B > gpurun_out/b2_rel2.json" \
 "120|b_acq2|CAPMI_LIB=$L/acqonly.so $B > gpurun_out/b2_acq2.json" \
 "120|b_mm2|$B > gpurun_out/b2_mm2.json" \
 "120|b_mm_noroute2|CAPMI_R4_ROUTE=0 $B > gpurun_out/b2_mm_noroute2.json"
