#!/bin/bash
# v5 (forced) vs the default kernels on config 4 (50 rows, T=1000) and config 2 (J=16).
mkdir -p gpurun_out
for v in 0 5; do
  SKELDIFF_GL_VARIANT=$v timeout -k 10 300 python -u bench.py --config h36m_t1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_v$v.log 2>&1
  rc=$?; echo "cfg4 v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/c4_v$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg4 v$v', round(r['value'],2))"
done
SKELDIFF_GL_VARIANT=5 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c2_v5.log 2>&1
rc=$?; echo "cfg2 v5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/c2_v5.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg2 v5', round(r['value'],1))"
