#!/bin/bash
# round 4: SQ counter passes on single GEMM launches (tools/r03/sq.sh's recipe), then the table
export CASES="${CASES:-l1c2:x3c l3c3:x3d l3c2:x3p l3c2:x3w l3c1:x3}"
bash tools/r03/sq.sh
