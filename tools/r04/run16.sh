#!/bin/bash
# round 4: x3d data-parallel instead of stream-K (CAPMI_SK_FAMILY_OFF=5) on the fine-tune config (its 1x1
# data gradients accumulate into C: 226 MB per launch) and on the headline, alternating arms
F="python bench.py --no-cpu-baseline --no-roofline --config glove_finetune"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "200|f0|$F > gpurun_out/b16_f0.json" \
 "200|f5|CAPMI_SK_FAMILY_OFF=5 $F > gpurun_out/b16_f5.json" \
 "200|f0b|$F > gpurun_out/b16_f0b.json" \
 "200|f5b|CAPMI_SK_FAMILY_OFF=5 $F > gpurun_out/b16_f5b.json" \
 "150|h0|$B > gpurun_out/b16_h0.json" \
 "150|h5|CAPMI_SK_FAMILY_OFF=5 $B > gpurun_out/b16_h5.json"
