#!/bin/bash
# full GPU suite (as the driver runs it) + smoke
tools/gpu_steps.sh \
  "900|t_all|python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread" \
  "120|smoke|python -c 'import __graft_entry__ as g; g.smoke()'"
