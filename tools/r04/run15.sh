#!/bin/bash
# round 4 closing measurement set: the three configs (bench line, kernel trace, FETCH / WRITE passes)
CFG=attention tools/r04/final_measure.sh && CFG=glove_finetune tools/r04/final_measure.sh && \
CFG=bert_attention tools/r04/final_measure.sh
