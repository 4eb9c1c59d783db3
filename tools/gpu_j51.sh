#!/bin/bash
# Config 3 (MANO J=51) per graph-linear generation: v1 vs v2 (the default fall-through).
mkdir -p gpurun_out
for v in 2 1; do
  SKELDIFF_GL_VARIANT=$v timeout -k 10 300 python -u bench.py --config mano51 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/j51_v$v.log 2>&1
  rc=$?; echo "v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/j51_v$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('v$v', round(r['value'],1), r['kernels_per_denoise_step_ms'])"
done
