#!/bin/bash
# Per-conv kernel times on single launches (tools/gemm_one.py) across arms: variant builds (ab/<name>.so from
# tools/abvar.sh) and / or environment settings, optionally with the in-kernel phase stamps (tools/stamps.py,
# a stamp build). One GPU step per arm (tools/gpu_steps.sh).
#   ARMS  = "name=ENV=1,ENV2=0 ..."  (an arm named base runs the in-tree library; CAPMI_LIB=ab/x.so picks a build)
#   CASES = "shape:flag,flag ..."    gemm_one.py shapes and flags (commas for spaces)
#   REPS (30), STAMPS=ab/stamp.so (run tools/stamps.py on the cases with that build too)
# e.g. ARMS="base= sk1=CAPMI_BF16_SK=1" CASES="l3c2:--bf16io l4c2:--bf16io" tools/shape_times.sh
# (the round-5 probe recipes r05_probe1..33 were instances of this: per-shape A/B of build flags and env arms)
REPS=${REPS:-30}
steps=()
for arm in ${ARMS:-base=}; do
  name=${arm%%=*}; envs=${arm#*=}; envs=${envs//,/ }
  cmd=""
  for c in $CASES; do sh=${c%%:*}; f=${c#*:}; [ "$f" = "$c" ] && f=""
    cmd="$cmd $envs python tools/gemm_one.py --reps $REPS --shape $sh ${f//,/ } &&"; done
  steps+=("300|t_$name|${cmd% &&}")
done
if [ -n "$STAMPS" ]; then
  cmd=""
  for c in $CASES; do sh=${c%%:*}; f=${c#*:}; [ "$f" = "$c" ] && f=""
    cmd="$cmd CAPMI_LIB=$STAMPS python tools/stamps.py --shape $sh ${f//,/ } &&"; done
  steps+=("300|stamps|${cmd% &&}")
fi
tools/gpu_steps.sh "${steps[@]}"
