#!/bin/bash
# fused BN finalize (capmi_bn_finalize_apply): kernel + encoder-level tests, then the A/B
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "400|t7|python -u -m pytest tests/test_gpu_bn_fused.py tests/test_gpu_x3.py tests/test_gpu_bf16.py tests/test_gpu_train_step.py tests/test_gpu_encoder.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "100|a_fuse|$B" "100|a_nofuse|CAPMI_BN_FUSE=0 $B" "100|a_fuse2|$B" "100|a_nofuse2|CAPMI_BN_FUSE=0 $B" \
  "100|c_fuse|$B --config bert_attention" "100|c_nofuse|CAPMI_BN_FUSE=0 $B --config bert_attention" \
  "100|c_fuse2|$B --config bert_attention" "100|c_nofuse2|CAPMI_BN_FUSE=0 $B --config bert_attention" \
  "100|a_fuse_b256|CAPMI_BNFA_BLOCKS=256 $B" "100|a_fuse_b1024|CAPMI_BNFA_BLOCKS=1024 $B"
for f in gpurun_out/a_*.log gpurun_out/c_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
