#!/bin/bash
# round 4: x3d two-deep pipeline under the planner's rule (parity first), the shorter-chain canonical BN finalize,
# then bench A/B: default / pipeline off / the round-3 direct finalize
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "300|x3t|$P tests/test_gpu_x3.py -k 'x3d or x3p or encoder_x3_matches'" \
 "300|x3t1|CAPMI_X3D_PIPE=1 $P tests/test_gpu_x3.py -k 'x3d'" \
 "200|bnf|$P tests/test_gpu_bn_final.py" \
 "120|b_d|$B > gpurun_out/b7_d.json" \
 "120|b_p0|CAPMI_X3D_PIPE=0 $B > gpurun_out/b7_p0.json" \
 "120|b_old|CAPMI_BNF_OLD=1 $B > gpurun_out/b7_old.json" \
 "120|b_d2|$B > gpurun_out/b7_d2.json" \
 "120|b_p02|CAPMI_X3D_PIPE=0 $B > gpurun_out/b7_p02.json" \
 "120|b_old2|CAPMI_BNF_OLD=1 $B > gpurun_out/b7_old2.json" \
 "200|b_ft|python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b7_ft.json"
