#!/bin/bash
# Training side: kernel parity tests, the training-step bench (HIP vs torch ops) at J = 16 / 21,
# and a kernel trace of the HIP step.
OUT=gpurun_out/train_r03c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_training.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_train.log 2>&1
rc=$?; echo "training tests rc=$rc: $(tail -1 $OUT/pytest_train.log)"; [ $rc -eq 0 ] || exit $rc
for J in 16 21; do
  timeout -k 10 300 python -u tools/bench_train.py --J $J --rows 1024 --steps 10 --warmup 3 > $OUT/train$J.json 2> $OUT/train$J.err
  rc=$?; echo "train J=$J rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/train$J.json'));print(round(d['hip']['ms_per_step'],2),'ms vs torch',round(d['torch_ops_same_gpu']['ms_per_step'],2),'ms speedup',round(d['speedup'],2))")"; [ $rc -eq 0 ] || exit $rc
done
bash tools/prof_train.sh && cp gpurun_out/prof_train/run_kernel_stats.csv $OUT/train_kernel_stats.csv
