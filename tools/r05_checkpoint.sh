#!/bin/bash
# round 5 checkpoint: the GPU suite, then the headline measurement set (bench line, kernel trace, FETCH / WRITE)
tools/gpu_steps.sh "900|suite|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/suite.log && ! grep -q " failed" gpurun_out/suite.log || exit 1
CFG=attention bash tools/final_measure.sh
