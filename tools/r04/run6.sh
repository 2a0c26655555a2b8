#!/bin/bash
# round 4: the direct 3x3 conv (x3c) parity first (short limits), the x3 / BN tests, per-conv times, then bench
# A/B: default / x3c off / x3d pipeline off / the round-3 direct finalize
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "200|x3c|$P tests/test_gpu_x3.py -k x3c" \
 "400|x3t|$P tests/test_gpu_x3.py tests/test_gpu_bn_final.py tests/test_gpu_encoder.py" \
 "200|x3c_t|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/x3c_time.txt" \
 "120|b_d|$B > gpurun_out/b8_d.json" \
 "120|b_c0|CAPMI_X3C=0 $B > gpurun_out/b8_c0.json" \
 "120|b_p0|CAPMI_X3D_PIPE=0 $B > gpurun_out/b8_p0.json" \
 "120|b_old|CAPMI_BNF_OLD=1 $B > gpurun_out/b8_old.json" \
 "120|b_d2|$B > gpurun_out/b8_d2.json" \
 "120|b_c02|CAPMI_X3C=0 $B > gpurun_out/b8_c02.json" \
 "120|b_p02|CAPMI_X3D_PIPE=0 $B > gpurun_out/b8_p02.json" \
 "120|b_old2|CAPMI_BNF_OLD=1 $B > gpurun_out/b8_old2.json" \
 "200|b_ft|python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b8_ft.json"
