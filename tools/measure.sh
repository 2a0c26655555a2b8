#!/bin/bash
# Measurement sets on one GPU box (each GPU step under its own time limit, tools/gpu_steps.sh):
#   tools/measure.sh suite                 the GPU test suite
#   tools/measure.sh lines                 suite, then the default bench line of every GPU config
#   tools/measure.sh final CFG [CFG ...]   per config: bench line, rocprofv3 kernel trace, FETCH / WRITE PMC passes
#                                          (tools/final_measure.sh)
#   tools/measure.sh checkpoint            suite, then `final attention`
# (round 5's r05_lines / r05_checkpoint / r05_final / r05_measure scripts, folded)
suite() {
  tools/gpu_steps.sh "900|suite|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || return $?
  grep -q " passed" gpurun_out/suite.log && ! grep -q " failed" gpurun_out/suite.log
}
lines() {
  tools/gpu_steps.sh "400|line_attention|python bench.py > gpurun_out/line_attention.json" \
    "400|line_glove_finetune|python bench.py --config glove_finetune > gpurun_out/line_glove_finetune.json" \
    "400|line_bert_attention|python bench.py --config bert_attention > gpurun_out/line_bert_attention.json"
}
final() {
  for c in "$@"; do CFG=$c bash tools/final_measure.sh || return $?; done
}
what=$1; shift
case "$what" in
  suite) suite ;;
  lines) suite && lines ;;
  final) final "$@" ;;
  checkpoint) suite && final attention ;;
  *) echo "usage: tools/measure.sh suite|lines|final CFG...|checkpoint" >&2; exit 2 ;;
esac
