#!/bin/bash
# Kernel trace of the HIP training step alone (tools/prof_train.sh).
OUT=gpurun_out/ab6_r03
mkdir -p $OUT
bash tools/prof_train.sh || exit $?
cp gpurun_out/prof_train/run_kernel_stats.csv $OUT/train_kernel_stats.csv
