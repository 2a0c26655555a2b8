#!/bin/bash
# L2 hit rate and memory-side reads of conv GEMM launches (tools/gemm_one.py) -- one rocprofv3 --pmc pass per case
# (TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum, each under its own kill timer), summarised by tools/pmc_l2.py into
# gpurun_out/l2_table.txt. CASES = "shape:flag,flag[:lib] ..." (default: the x3 family at its bench shapes)
R=$GRAFT_REPO_ROOT
CASES=${CASES:-"l3c2:--x3p l3c3:--x3d,--dense l3c1:--x3 l2c2:--x3p"}
mkdir -p $R/gpurun_out/l2
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  IFS=: read -r sh f lib <<< "$c"
  f=${f//,/ }
  CAPMI_LIB=${lib:+$R/$lib} timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
    -d $R/gpurun_out/l2/$sh${f// /}${lib:+_$(basename $lib .so)} -o pmc -- python $R/tools/gemm_one.py --shape $sh --reps 5 $f \
    > /dev/null 2>&1 || exit 1
done
cd $R && python tools/pmc_l2.py gpurun_out/l2 > gpurun_out/l2_table.txt && rm -rf gpurun_out/l2 && cat gpurun_out/l2_table.txt
