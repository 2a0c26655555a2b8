#!/bin/bash
# SQ counters of single conv GEMMs (fp32 and bf16) + plain timings. Output under gpurun_out/pmcconv/.
R=$GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
mkdir -p gpurun_out/pmcconv
for sh in l3c2 l3c3 l3c1; do
  for bf in "" "--bf16"; do
    timeout -k 10 60 python tools/gemm_one.py --shape $sh $bf >> gpurun_out/pmcconv/times.txt 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for sh in l3c2 l3c3; do
  for bf in "" "--bf16"; do
    timeout -s KILL 60 rocprofv3 --pmc $C -d $R/gpurun_out/pmcconv/$sh$bf -o pmc -- python $R/tools/gemm_one.py --shape $sh --reps 5 $bf > /dev/null 2>&1 || exit 1
  done
done
