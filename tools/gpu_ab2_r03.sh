#!/bin/bash
# XCD-aligned k_gl4t / MODE 2 block mapping (SKELDIFF_XCD_ALIGN): bitwise route
# tests with it on, same-box config-2 A/B (1 and 3 chains, alternated), PMC traffic with it on.
OUT=gpurun_out/xcd_r03
mkdir -p $OUT
SKELDIFF_XCD_ALIGN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tiled_split_route_bitwise or config2_as_benched or share_cus or shard" > $OUT/pytest.log 2>&1
rc=$?; echo "aligned tests rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for E in 0 1; do
    SKELDIFF_XCD_ALIGN=$E SWEEP_ROUTES=0 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16 > $OUT/s.log 2>&1
    rc=$?; echo "XCD_ALIGN=$E rc=$rc: $(grep '^{' $OUT/s.log | python3 -c "import json,sys; print(' '.join(f\"c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  done
done
SKELDIFF_XCD_ALIGN=1 bash tools/prof_bench.sh r03x
