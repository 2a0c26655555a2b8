#!/bin/bash
# round 4: x3w kernel tests first, then the GPU suite (one process), smoke, then bench arms
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "300|x3w|python -u -m pytest tests/test_gpu_finetune.py -k x3w -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "900|suite|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -s" \
 "200|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "120|b_route|$B > gpurun_out/b3_route.json" \
 "120|b_noroute|CAPMI_R4_ROUTE=0 $B > gpurun_out/b3_noroute.json" \
 "120|b_route2|$B > gpurun_out/b3_route2.json" \
 "120|b_noroute2|CAPMI_R4_ROUTE=0 $B > gpurun_out/b3_noroute2.json" \
 "200|b_ft|python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b3_ft.json" \
 "200|b_ft_nts|CAPMI_FT_WGRAD_X3W=0 python bench.py --no-cpu-baseline --no-roofline --config glove_finetune > gpurun_out/b3_ft_nts.json"
