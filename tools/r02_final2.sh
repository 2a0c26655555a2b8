#!/bin/bash
# round-2 closing set after the fine-tune x3d dgrads: full GPU suite, smoke, fine-tune line (with
# the PMC traffic of its own run now in profiles/), headline line
tools/gpu_steps.sh "700|gpu_all|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" && \
tools/gpu_steps.sh "200|smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|bench_ft|python bench.py --config glove_finetune --no-cpu-baseline" \
  "300|bench_default|python bench.py"
