#!/bin/bash
# round 5, probe 6: bench A/B with the roofline pass (per-kernel conv timing) on base / p2 / v2
B="python bench.py --no-cpu-baseline"
tools/gpu_steps.sh \
  "200|b6_base1|$B > gpurun_out/b6_base1.json" \
  "200|b6_p2_1|CAPMI_LIB=ab/p2.so $B > gpurun_out/b6_p2_1.json" \
  "200|b6_v2_1|CAPMI_LIB=ab/v2.so $B > gpurun_out/b6_v2_1.json" \
  "200|b6_base2|$B > gpurun_out/b6_base2.json" \
  "200|b6_p2_2|CAPMI_LIB=ab/p2.so $B > gpurun_out/b6_p2_2.json" \
  "200|b6_v2_2|CAPMI_LIB=ab/v2.so $B > gpurun_out/b6_v2_2.json"
