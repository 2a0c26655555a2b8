#!/bin/bash
# round 5 measurement set: final_measure.sh for the given configs, one after the other (stops at the first failure)
for c in "$@"; do CFG=$c bash tools/final_measure.sh || exit $?; done
