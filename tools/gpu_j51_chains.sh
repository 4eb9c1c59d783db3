#!/bin/bash
# Config 3 (MANO J=51, v5) at 1, 2, 3 row chains.
mkdir -p gpurun_out
for c in 1 2 3; do
  SKELDIFF_CHAINS=$c timeout -k 10 300 python -u bench.py --config mano51 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/j51_c$c.log 2>&1
  rc=$?; echo "chains $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/j51_c$c.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('chains $c', round(r['value'],1))"
done
