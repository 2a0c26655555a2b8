#!/bin/bash
# round 5, probe 31: the in-kernel clock and per-phase cycles of the bench's x3p and x3d instantiations at the closing
# code (stamp build ab/stamp.so; tools/stamps.py), VERDICT r4 item 3's clock re-take
S="python tools/stamps.py"
tools/gpu_steps.sh "200|stamps31|CAPMI_LIB=ab/stamp.so $S --shape l3c2 --x3p && CAPMI_LIB=ab/stamp.so $S --shape l2c2 --x3p && CAPMI_LIB=ab/stamp.so $S --shape l3c3 --x3d --dense"
