#!/bin/bash
# k_gl4t with the next tile's weight fragments read ahead of the current tile's MFMAs (this build)
# vs the previous build (libskeldiff_old.so): route tests, then a same-box A/B alternated twice.
OUT=gpurun_out/pipe_r03
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tiled_split_route_bitwise or config2_as_benched or share_cus" > $OUT/pytest.log 2>&1
rc=$?; echo "route tests rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export SKELDIFF_LIB=$PWD/skeletondiffusion_amd/libskeldiff_old.so; else unset SKELDIFF_LIB; fi
    SWEEP_ROUTES=0 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16 freeman17 > $OUT/s.log 2>&1
    rc=$?; echo "$L rc=$rc: $(grep '^{' $OUT/s.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}/c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  done
done
