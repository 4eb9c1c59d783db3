#!/bin/bash
# rocprofv3 kernel trace of config 3 (MANO J=51, v5 graph-linears), T=4.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_j51
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_j51 -o run -- \
    python3 bench.py --config mano51 --T 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_j51/log.txt 2>&1
rc=$?; echo "prof_rc=$rc"; exit $rc
