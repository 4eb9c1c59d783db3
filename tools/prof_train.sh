#!/bin/bash
# rocprofv3 kernel trace of the training-step bench (HIP graph-linears only).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- \
    python3 tools/bench_train.py --J ${J:-16} --rows 1024 --steps 3 --warmup 1 --modes hip > gpurun_out/prof_train/log.txt 2>&1
rc=$?; echo "prof_rc=$rc"; exit $rc
