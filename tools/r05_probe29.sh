#!/bin/bash
# round 5, probe 29: BN finalize / backward finalize with every slice load in flight (in-tree) vs the round-4 loops
# (ab/old.so): their bit-exact tests, the finalize alone per shape, the three configs alternating
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
tools/gpu_steps.sh "300|bnf_tests|$T tests/test_gpu_bn_final.py tests/test_gpu_finetune.py -k 'bn_ or finalize or bn_backward'" || exit $?
grep -q " passed" gpurun_out/bnf_tests.log && ! grep -q " failed" gpurun_out/bnf_tests.log || exit 1
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "120|bnf_new|python tools/bnf_time.py" "120|bnf_old|CAPMI_LIB=ab/old.so python tools/bnf_time.py" \
  "200|h1|$B" "200|h0|CAPMI_LIB=ab/old.so $B" "200|h1b|$B" "200|h0b|CAPMI_LIB=ab/old.so $B" \
  "200|c1|$B --config bert_attention" "200|c0|CAPMI_LIB=ab/old.so $B --config bert_attention" \
  "200|f1|$B --config glove_finetune" "200|f0|CAPMI_LIB=ab/old.so $B --config glove_finetune"
for f in h1 h0 h1b h0b c1 c0 f1 f0; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
