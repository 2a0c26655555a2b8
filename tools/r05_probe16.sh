#!/bin/bash
# round 5, probe 16: x3p with the LDS-DMA issued by loader waves only (X3P_LOADERS = 4, 2) vs every wave
tools/gpu_steps.sh "300|ld_ab|python tools/ab_inproc.py --libs base,ab/ld4.so,ab/ld2.so --cases \"l3c2:--x3p l2c2:--x3p l4c2:--x3p\" --rounds 7"
