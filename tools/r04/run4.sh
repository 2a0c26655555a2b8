#!/bin/bash
# round 4: the pipelined x3d / x3w (parity tests first, short limits), per-conv and per-wgrad timing, the canonical
# BN finalize (test, bench A/B against the round-3 direct kernel), x3d pipeline A/B, the fine-tune bench
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
NP="CAPMI_LIB=$PWD/ab/nopipe.so"
tools/gpu_steps.sh \
 "300|x3t|$P tests/test_gpu_x3.py -k 'x3d or x3p or encoder_x3_matches'" \
 "300|x3w|$P tests/test_gpu_finetune.py -k x3w" \
 "200|bnf|$P tests/test_gpu_bn_final.py" \
 "200|x3wt|python -u tools/r04/x3w_debug.py > gpurun_out/x3w_debug2.txt" \
 "200|conv|python -u tools/r03/conv_ab.py --arms x3,x3d,x3p > gpurun_out/conv_pipe.md" \
 "200|conv_np|$NP python -u tools/r03/conv_ab.py --arms x3d > gpurun_out/conv_nopipe.md" \
 "120|b_new|$B > gpurun_out/b6_new.json" \
 "120|b_np|$NP $B > gpurun_out/b6_np.json" \
 "120|b_old|CAPMI_BNF_OLD=1 $B > gpurun_out/b6_old.json" \
 "120|b_new2|$B > gpurun_out/b6_new2.json" \
 "120|b_np2|$NP $B > gpurun_out/b6_np2.json" \
 "120|b_old2|CAPMI_BNF_OLD=1 $B > gpurun_out/b6_old2.json" \
 "200|b_ft|python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b6_ft.json" \
 "200|b_ft_np|$NP python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b6_ft_np.json"
