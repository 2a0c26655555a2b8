#!/bin/bash
# round 4: x3c with the LDS-only tap barrier (parity, timing); where x3p's l3c2 time goes -- data-parallel (98 workgroups, one tile each) against stream-K on 256 /
# 196 / 98 CUs; then the bench with stream-K grids sized below the CU count (CUs left to the decoder stream)
G="python -u tools/gemm_one.py --shape l3c2 --x3p --reps 50"
B="python bench.py --no-cpu-baseline --no-roofline"
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
tools/gpu_steps.sh \
 "200|x3c|$P tests/test_gpu_x3.py -k 'x3c or encoder_x3_matches'" \
 "120|x3c_t|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/x3c_time5.txt" \
 "120|sk256|$G > gpurun_out/sk_256.txt" \
 "120|skoff|CAPMI_SK_OFF=1 $G > gpurun_out/sk_off.txt" \
 "120|sk196|CAPMI_SK_CUS=196 $G > gpurun_out/sk_196.txt" \
 "120|sk98|CAPMI_SK_CUS=98 $G > gpurun_out/sk_98.txt" \
 "120|nohyb|CAPMI_SK_HYBRID=0 $G > gpurun_out/sk_nohyb.txt" \
 "120|l3c3|python -u tools/gemm_one.py --shape l3c3 --x3d --reps 50 > gpurun_out/l3c3_x3d.txt" \
 "120|l3c3off|CAPMI_SK_OFF=1 python -u tools/gemm_one.py --shape l3c3 --x3d --reps 50 > gpurun_out/l3c3_x3d_off.txt" \
 "150|b0|$B > gpurun_out/b11_0.json" \
 "150|b224|CAPMI_SK_CUS=224 $B > gpurun_out/b11_224.json" \
 "150|b192|CAPMI_SK_CUS=192 $B > gpurun_out/b11_192.json" \
 "150|b0b|$B > gpurun_out/b11_0b.json" \
 "150|b224b|CAPMI_SK_CUS=224 $B > gpurun_out/b11_224b.json" \
 "150|b192b|CAPMI_SK_CUS=192 $B > gpurun_out/b11_192b.json"
