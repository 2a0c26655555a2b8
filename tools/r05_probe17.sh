#!/bin/bash
# round 5, probe 17: where config 5's bf16 GEMM spends its time (timing-only builds: no C stores / no MFMAs / no
# operand loads), and the persistent grid
tools/gpu_steps.sh "200|bf16_skip|python tools/ab_inproc.py --libs base,ab/bsk1.so,ab/bsk2.so,ab/bsk4.so --cases \"l3c3:--bf16io l3c2:--bf16io l4c3:--bf16io\" --rounds 5" \
  "200|bf16_persist|python tools/r05_probe17.py"
