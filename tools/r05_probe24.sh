#!/bin/bash
# round 5, probe 24: spatial partition of the pipelined step -- decoder stream on n CUs, encoder stream (and its
# stream-K grids, CAPMI_SK_CUS) on the rest, two CU-masked HIP streams (CAPMI_PIPE_CUMASK) vs the default
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline"
a=()
for r in 1 2; do
  a+=("200|base$r|$B")
  a+=("200|m32s$r|CAPMI_PIPE_CUMASK=32:s CAPMI_SK_CUS=224 $B")
  a+=("200|m32t$r|CAPMI_PIPE_CUMASK=32 CAPMI_SK_CUS=224 $B")
  a+=("200|m64s$r|CAPMI_PIPE_CUMASK=64:s CAPMI_SK_CUS=192 $B")
  a+=("200|m16s$r|CAPMI_PIPE_CUMASK=16:s CAPMI_SK_CUS=240 $B")
done
tools/gpu_steps.sh "${a[@]}"
for f in base m32s m32t m64s m16s; do for r in 1 2; do echo "$f$r $(grep -o '"value": [0-9.]*' gpurun_out/$f$r.log)"; done; done
