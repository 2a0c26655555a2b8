#!/bin/bash
# round 4: the fine-tune and bert measurement sets (bench line, kernel trace, FETCH / WRITE passes)
CFG=glove_finetune tools/r04/final_measure.sh && CFG=bert_attention tools/r04/final_measure.sh
