#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) on single conv GEMMs: VARIANTS from
# native (fp32 MFMA), x3, x3p; SHAPES from tools/gemm_one.py. Output: gpurun_out/pmcx3/<shape>-<variant>_p<pass>/
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"
mkdir -p gpurun_out/pmcx3
cd /tmp && export TMPDIR=/tmp
for sh in ${SHAPES:-l3c2}; do
  for v in ${VARIANTS:-native x3}; do
    flag=""
    [ "$v" != native ] && flag="--$v"
    n=1
    for C in "$P1" "$P2"; do
      timeout -s KILL 60 rocprofv3 --pmc $C -d $R/gpurun_out/pmcx3/$sh-${v}_p$n -o pmc -- python $R/tools/gemm_one.py --shape $sh --reps 5 $flag > /dev/null 2>&1 || exit 1
      n=$((n+1))
    done
  done
done
cd $R && python tools/pmc_table.py gpurun_out/pmcx3 > gpurun_out/pmcx3_table.txt && rm -rf gpurun_out/pmcx3
