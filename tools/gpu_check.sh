#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> short bench.  Stops at the first crash-type
# exit (fault/abort/segfault/timeout); a plain test failure (rc 1) still lets the bench run.
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; exit $rc
