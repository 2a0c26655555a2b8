#!/bin/bash
# round 5, probe 21: bf16 GEMM with the one-stage 128x64 form for K <= 256 (base) vs the round-4 library (old) and
# 5 waves / SIMD (w5); bf16 tests; config 5 bench on each library
c="l3c3:--bf16io l2c3:--bf16io l1c3:--bf16io l1c1:--bf16io ds1:--bf16io l4c3:--bf16io l3c1:--bf16io"
tools/gpu_steps.sh "300|bf16io_tests|python -u -m pytest tests/test_gpu_bf16io.py -x -q --timeout 120 --timeout-method thread" \
  "200|bf16_ab|python tools/ab_inproc.py --libs base,ab/old.so,ab/w5.so --cases \"$c\" --rounds 5" \
  "300|bench_new|python bench.py --config bert_attention --steps 30 --warmup 5 --no-cpu-baseline --no-roofline" \
  "300|bench_old|CAPMI_LIB=ab/old.so python bench.py --config bert_attention --steps 30 --warmup 5 --no-cpu-baseline --no-roofline" \
  "300|bench_new2|python bench.py --config bert_attention --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
