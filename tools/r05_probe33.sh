#!/bin/bash
# round 5, probe 33: config 5 with 128x64 bf16 tiles on grids that fill at most half the CUs (in-tree) vs before
# (ab/old.so): the bf16 tests, per-shape times, config 5 alternating
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python bench.py --config bert_attention --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "300|bf16_tests|$T tests/test_gpu_bf16io.py tests/test_gpu_bench_paths.py -k 'bf16 or config5 or bert'" || exit $?
grep -q " passed" gpurun_out/bf16_tests.log && ! grep -q " failed" gpurun_out/bf16_tests.log || exit 1
tools/gpu_steps.sh "200|n1|$B" "200|n0|CAPMI_LIB=ab/old.so $B" "200|n1b|$B" "200|n0b|CAPMI_LIB=ab/old.so $B"
for f in n1 n0 n1b n0b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
