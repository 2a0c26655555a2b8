#!/bin/bash
# round 5, probe 18: config 5's bf16 GEMM with the LDS-staged 16-B store epilogue (base) vs the 2-B store one
# (epi0) and vs no C stores (bsk1); then data-parallel vs persistent grid on the new epilogue
tools/gpu_steps.sh "200|bf16_epi|python tools/ab_inproc.py --libs base,ab/epi0.so,ab/bsk1.so --cases \"l3c3:--bf16io l3c2:--bf16io l4c3:--bf16io l2c3:--bf16io l1c3:--bf16io l3c1:--bf16io\" --rounds 5" \
  "200|bf16_persist|python tools/r05_probe17.py"
