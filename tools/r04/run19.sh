#!/bin/bash
# round 4: beta epilogues with batched C loads (data-parallel x3d for beta problems) -- parity, then the
# fine-tune bench against CAPMI_X3D_BETA_SK=1, and the headline
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python bench.py --no-cpu-baseline --no-roofline"
tools/gpu_steps.sh \
 "600|t|$P tests/test_gpu_finetune.py tests/test_gpu_x3.py tests/test_gpu_gemm.py tests/test_gpu_split_gemm.py" \
 "200|f1|$B --config glove_finetune > gpurun_out/b19_f1.json" \
 "200|fs|CAPMI_X3D_BETA_SK=1 $B --config glove_finetune > gpurun_out/b19_fs.json" \
 "200|f2|$B --config glove_finetune > gpurun_out/b19_f2.json" \
 "200|fs2|CAPMI_X3D_BETA_SK=1 $B --config glove_finetune > gpurun_out/b19_fs2.json" \
 "150|h1|$B > gpurun_out/b19_h1.json" \
 "150|h2|$B > gpurun_out/b19_h2.json"
