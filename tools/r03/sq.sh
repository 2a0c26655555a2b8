#!/bin/bash
# SQ counter passes (two rocprofv3 runs per case, each under its own kill timer) on single conv GEMMs:
# CASES = "shape:variant ..." (variant: x3 / x3d / x3p / x3s / native; tools/gemm_one.py shapes).
# Output: gpurun_out/sq_table.txt (tools/pmc_table.py) and the raw dbs under gpurun_out/pmcx3/.
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"
mkdir -p $R/gpurun_out/pmcx3
cd /tmp && export TMPDIR=/tmp
for c in ${CASES:-l3c3:x3d l3c2:x3p l3c1:x3 l1c3:x3 l1c2:x3}; do
  sh=${c%%:*}; v=${c##*:}
  flag=""
  [ "$v" != native ] && flag="--$v"
  timeout -k 10 60 python $R/tools/gemm_one.py --shape $sh --reps 20 $flag >> $R/gpurun_out/sq_times.txt 2>&1 || exit 1
  n=1
  for C in "$P1" "$P2"; do
    timeout -s KILL 60 rocprofv3 --pmc $C -d $R/gpurun_out/pmcx3/$sh-${v}_p$n -o pmc -- python $R/tools/gemm_one.py --shape $sh --reps 5 $flag > /dev/null 2>&1 || exit 1
    n=$((n+1))
  done
done
cd $R && python tools/pmc_table.py gpurun_out/pmcx3 > gpurun_out/sq_table.txt && rm -rf gpurun_out/pmcx3
