#!/bin/bash
# round 5 closing run on one box: probe 30 (weight-batch tests, config 4 A/B, trace), the GPU suite and the three
# bench lines (r05_lines.sh), config 4's trace + PMC passes (final_measure.sh)
tools/r05_probe30.sh || exit $?
grep -q " passed" gpurun_out/ft_tests.log && ! grep -q " failed" gpurun_out/ft_tests.log || exit 1
tools/r05_lines.sh || exit $?
CFG=glove_finetune bash tools/final_measure.sh
