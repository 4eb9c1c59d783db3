#!/bin/bash
# MANO mixing pass: 4 / 8 rows per k_gl5_mixm workgroup (SKELDIFF_V5_ROWS), same box, alternated.
OUT=gpurun_out/mix4_r03
mkdir -p $OUT
timeout -k 10 300 env SKELDIFF_V5_ROWS=4 python -u -m pytest tests/test_gpu_v5.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "v5 tests (4 rows) rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for R in 8 4; do
    SKELDIFF_V5_ROWS=$R SWEEP_ROUTES=0 SWEEP_CHAINS=3 timeout -k 10 300 python -u tools/sweep_routes.py mano51 > $OUT/s.log 2>&1
    rc=$?; echo "V5_ROWS=$R rc=$rc: $(grep '^{' $OUT/s.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  done
done
