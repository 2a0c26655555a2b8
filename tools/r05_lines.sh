#!/bin/bash
# round 5: the GPU suite, then the default bench line of every config (one box)
tools/gpu_steps.sh "900|suite|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/suite.log && ! grep -q " failed" gpurun_out/suite.log || exit 1
tools/gpu_steps.sh "400|line_attention|python bench.py > gpurun_out/line_attention.json" \
  "400|line_glove_finetune|python bench.py --config glove_finetune > gpurun_out/line_glove_finetune.json" \
  "400|line_bert_attention|python bench.py --config bert_attention > gpurun_out/line_bert_attention.json"
