#!/bin/bash
# round 4: the x3d pipeline everywhere (CAPMI_X3D_PIPE=1) against the per-conv rule, headline and fine-tune
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "120|p1|CAPMI_X3D_PIPE=1 $B > gpurun_out/b26_p1.json" \
 "120|d1|$B > gpurun_out/b26_d1.json" \
 "120|p2|CAPMI_X3D_PIPE=1 $B > gpurun_out/b26_p2.json" \
 "120|d2|$B > gpurun_out/b26_d2.json" \
 "200|fp|CAPMI_X3D_PIPE=1 $B --config glove_finetune > gpurun_out/b26_fp.json" \
 "200|fd|$B --config glove_finetune > gpurun_out/b26_fd.json"
