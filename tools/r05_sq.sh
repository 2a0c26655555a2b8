#!/bin/bash
# round 5: SQ passes (tools/sq.sh) on the exact instantiations the benches run, one case per kernel family:
# x3p 3x3, x3d dense-row prologue, gemm_x3<128,0>, x3c, x3s, x3w, the bf16 GEMM (config 5) in both forms
CASES="l3c2:--x3p l3c3:--x3d,--dense l3c1:--x3 l1c2:--x3c l1c3:--x3s l3c2:--x3w l3c3:--bf16io l3c2:--bf16io" bash tools/sq.sh
