#!/bin/bash
# round 5, probe 20: BN backward launch shapes (BNB_V2 vs round 4) and the one-stage bf16 GEMM (probe 19)
tools/gpu_steps.sh "200|bnb|python tools/bnb_time.py --libs base,ab/bnb0.so" && tools/r05_probe19.sh
