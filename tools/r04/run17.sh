#!/bin/bash
# round 4 closing: the whole GPU suite and smoke() at the closing code
tools/gpu_steps.sh \
 "1000|suite|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "300|smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'"
