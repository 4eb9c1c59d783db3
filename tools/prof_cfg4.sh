#!/bin/bash
# rocprofv3 kernel trace of config 4 (one sequence x 50 futures, J=16), T=50.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_cfg4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg4 -o run -- \
    python3 bench.py --config h36m_t1000 --T 50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cfg4/log.txt 2>&1
rc=$?; echo "prof_rc=$rc"; exit $rc
