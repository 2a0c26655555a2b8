#!/bin/bash
# round 4: the wide direct conv (x3cw) -- parity first (short limit), then layer3 / layer2 timing against x3p
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
tools/gpu_steps.sh \
 "200|x3cw|$P tests/test_gpu_x3.py -k 'x3c'" \
 "60|w_l3|python -u tools/gemm_one.py --shape l3c2 --x3c --reps 50 > gpurun_out/w_l3c2.txt" \
 "60|w_l2|python -u tools/gemm_one.py --shape l2c2 --x3c --reps 50 > gpurun_out/w_l2c2.txt" \
 "60|p_l3|python -u tools/gemm_one.py --shape l3c2 --x3p --reps 50 > gpurun_out/p_l3c2.txt" \
 "60|p_l2|python -u tools/gemm_one.py --shape l2c2 --x3p --reps 50 > gpurun_out/p_l2c2.txt"
