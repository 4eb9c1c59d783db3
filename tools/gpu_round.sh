#!/bin/bash
# One GPU session: the GPU test suite, then the route / row-chain sweep (tools/sweep_routes.py).
# usage: bash tools/gpu_round.sh <tag> [sweep args...]
TAG=${1:-r03}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/sweep_routes.py "$@" > $OUT/sweep.log 2>&1
rc=$?
echo "sweep rc=$rc"
grep BEST $OUT/sweep.log
exit $rc
