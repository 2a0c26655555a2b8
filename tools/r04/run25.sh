#!/bin/bash
# round 4: env-knob A/B at the closing code (headline): x3d pipeline everywhere, column-major x3p tile order
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "120|d1|$B > gpurun_out/b25_d1.json" \
 "120|p1|CAPMI_X3D_PIPE=1 $B > gpurun_out/b25_p1.json" \
 "120|c1|CAPMI_X3P_ORDER=col $B > gpurun_out/b25_c1.json" \
 "120|d2|$B > gpurun_out/b25_d2.json" \
 "120|p2|CAPMI_X3D_PIPE=1 $B > gpurun_out/b25_p2.json" \
 "120|c2|CAPMI_X3P_ORDER=col $B > gpurun_out/b25_c2.json"
