#!/bin/bash
# round 4: the padded-band x3c (parity first, then timing), then the attention measurement set
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -s"
tools/gpu_steps.sh \
 "200|x3c|$P tests/test_gpu_x3.py -k 'x3c or encoder_x3_matches'" \
 "200|x3c_t|python -u tools/gemm_one.py --shape l1c2 --x3c --reps 50 > gpurun_out/x3c_time4.txt" || exit $?
CFG=attention tools/r04/final_measure.sh
