#!/bin/bash
# quick GPU iteration: parity/kernel tests -> GL microbench variants -> end-to-end bench
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_parity.py} -m gpu -q -x > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -le 1 ] || exit $rc
: > gpurun_out/bench_gl.log
for v in ${GL_VARIANTS:-"SKELDIFF_GL_VARIANT=0"}; do
  env $v timeout -k 10 120 python tools/bench_gl.py >> gpurun_out/bench_gl.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench_gl $v rc=$rc"; exit $rc; }
done
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/bench_q.log 2>&1
echo "bench_rc=$?"
