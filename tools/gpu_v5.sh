#!/bin/bash
# v5 graph-linear: kernel tests + J=51 sampler parity, then config 3 (MANO J=51) bench v5 vs v2.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "graph_linear or mano51 or 51" > gpurun_out/pytest_v5.log 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in 0 2; do
  SKELDIFF_GL_VARIANT=$v timeout -k 10 300 python -u bench.py --config mano51 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/j51_v$v.log 2>&1
  rc=$?; echo "v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/j51_v$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('v$v', round(r['value'],1), r['kernels_per_denoise_step_ms'])"
done
