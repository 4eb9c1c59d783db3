#!/bin/bash
# k_gl4t K = 192 forms on config 2: per-chunk weight stage shared by 4 waves (default) vs 8 waves
# (SKELDIFF_GL4T_CFG=5); bitwise route tests with 5, then a same-box A/B, alternated twice.
OUT=gpurun_out/gl4t5_r03
mkdir -p $OUT
SKELDIFF_GL4T_CFG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tiled_split_route_bitwise or config2_as_benched" > $OUT/pytest.log 2>&1
rc=$?; echo "cfg1 tests rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for C in 0 1; do
    SKELDIFF_GL4T_CFG=$C SWEEP_ROUTES=0 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16 > $OUT/s.log 2>&1
    rc=$?; echo "GL4T_CFG=$C rc=$rc: $(grep '^{' $OUT/s.log | python3 -c "import json,sys; print(' '.join(f\"c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  done
done
