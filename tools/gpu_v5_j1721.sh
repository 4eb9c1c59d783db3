#!/bin/bash
# v5 (forced) vs default (v4) on J=21 (AMASS) and J=17 (FreeMan), T=100, 3200 rows.
mkdir -p gpurun_out
for cfg in amass21 freeman17; do
  for v in 0 5; do
    SKELDIFF_GL_VARIANT=$v timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${cfg}_v$v.log 2>&1
    rc=$?; echo "$cfg v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep '^{' gpurun_out/${cfg}_v$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$cfg v$v', round(r['value'],1), r['kernels_per_denoise_step_ms'])"
  done
done
