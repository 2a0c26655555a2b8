#!/bin/bash
# SQ counter passes on single conv GEMM launches: two rocprofv3 --pmc runs per case (8 SQ + GRBM counters each,
# every run under its own kill timer), summarised by tools/pmc_table.py into gpurun_out/sq_table.txt.
# CASES = "shape:flag,flag[:lib] ..." -- a tools/gemm_one.py shape, its flags (commas for spaces) and optionally a
# variant build (CAPMI_LIB), e.g. CASES="l3c3:--x3d,--dense l3c2:--x3p:ab/p2.so" tools/sq.sh
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"
mkdir -p $R/gpurun_out/pmcx3
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  IFS=: read -r sh flags lib <<< "$c"
  f=${flags//,/ }
  if [ -n "$lib" ]; then export CAPMI_LIB=$R/$lib; else unset CAPMI_LIB; fi
  tag="$sh${flags//,/}${lib:+-$(basename $lib .so)}"; tag=${tag//--/-}
  timeout -k 10 60 python $R/tools/gemm_one.py --shape $sh --reps 20 $f >> $R/gpurun_out/sq_times.txt 2>&1 || exit 1
  n=1
  for C in "$P1" "$P2"; do
    timeout -s KILL 60 rocprofv3 --pmc $C -d $R/gpurun_out/pmcx3/${tag}_p$n -o pmc -- python $R/tools/gemm_one.py --shape $sh --reps 5 $f > /dev/null 2>&1 || exit 1
    n=$((n+1))
  done
done
cd $R && python tools/pmc_table.py gpurun_out/pmcx3 > gpurun_out/sq_table.txt && rm -rf gpurun_out/pmcx3
