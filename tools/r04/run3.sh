#!/bin/bash
# round 4: fused BN finalize -- its tests first (a spin bug would hang: short limit), then the x3 / encoder tests,
# the bench A/B (fused vs a finalize launch per BN), the fine-tune bench and the B = 64 parity tests
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "240|bnf|$P tests/test_gpu_bn_final.py" \
 "400|x3enc|$P tests/test_gpu_x3.py tests/test_gpu_encoder.py tests/test_gpu_gemm.py" \
 "120|b_bnf|$B > gpurun_out/b5_bnf.json" \
 "120|b_nobnf|CAPMI_BN_FUSED=0 $B > gpurun_out/b5_nobnf.json" \
 "120|b_bnf2|$B > gpurun_out/b5_bnf2.json" \
 "120|b_nobnf2|CAPMI_BN_FUSED=0 $B > gpurun_out/b5_nobnf2.json" \
 "200|b_ft|python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b5_ft.json" \
 "200|b_ft0|CAPMI_BN_FUSED=0 python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b5_ft0.json" \
 "600|flips|python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -s tests/test_gpu_headline_parity.py tests/test_gpu_bench_paths.py"
