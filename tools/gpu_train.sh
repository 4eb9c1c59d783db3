#!/bin/bash
# Training-side graph-linear on the GPU: its tests, the training-step bench (J=16, 21), and a
# rocprofv3 kernel trace of the J=16 bench (PROF=1).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_training.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_train.py --J 16 --rows 1024 > gpurun_out/bench_train16.log 2>&1
rc=$?; echo "bench16_rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_train.py --J 21 --rows 1024 > gpurun_out/bench_train21.log 2>&1
rc=$?; echo "bench21_rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = "1" ]; then bash tools/prof_train.sh; fi
