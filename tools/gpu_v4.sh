#!/bin/bash
# v4 iteration: GL kernel numerics, per-shape microbench per tile (CFGS), sampler parity + bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v4_kernels.log 2>&1
rc=$?; echo "kernels_rc=$rc"; tail -3 gpurun_out/v4_kernels.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-0 1 2}; do
  SKELDIFF_GL_VARIANT=4 SKELDIFF_GL4_CFG=$cfg timeout -k 10 120 python -u tools/bench_gl.py >> gpurun_out/v4_gl.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
grep -v amdgpu gpurun_out/v4_gl.log
[ "${FULL:-1}" = "1" ] || exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v4_pytest.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/v4_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v4_bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/v4_bench.log; exit $rc
