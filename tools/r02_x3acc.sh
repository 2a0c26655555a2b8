#!/bin/bash
# x3 shallow fine-tune accuracy under route variants (prints the aggregate gradient error)
T="timeout -k 10 200 python -u -m pytest tests/test_gpu_finetune.py -x -q -s --timeout 180 --timeout-method thread -k 'shallow_tight and x3'"
tools/gpu_steps.sh "220|a_def|$T" "220|a_nox3d|CAPMI_X3D=0 $T" "220|a_bwd32|CAPMI_FT_DGRAD_X3=0 CAPMI_FT_WGRAD_X3=0 $T" \
  "220|a_nox3d_bwd32|CAPMI_X3D=0 CAPMI_FT_DGRAD_X3=0 CAPMI_FT_WGRAD_X3=0 $T"
for f in gpurun_out/a_*.log; do echo "$f $(grep -o 'x3 shallow: .*' $f)"; done
