#!/bin/bash
# pipelined-step interference A/B: stream-K grids sized below the CU count (CAPMI_SK_CUS) and
# fewer, longer per-timestep decoder workgroups (CAPMI_DEC_WGS); then the measurement set
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh "120|ab_base|$B" "120|ab_dw128|CAPMI_DEC_WGS=128 $B" "120|ab_dw64|CAPMI_DEC_WGS=64 $B" \
  "120|ab_sk240|CAPMI_SK_CUS=240 $B" "120|ab_sk224|CAPMI_SK_CUS=224 $B" "120|ab_sk240_dw64|CAPMI_SK_CUS=240 CAPMI_DEC_WGS=64 $B" \
  "120|ab_base2|$B" "120|ab_bert|$B --config bert_attention" "120|ab_bert_sk240|CAPMI_SK_CUS=240 $B --config bert_attention" \
  "120|ab_bert_dw64|CAPMI_DEC_WGS=64 $B --config bert_attention"
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
