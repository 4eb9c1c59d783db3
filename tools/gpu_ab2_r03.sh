#!/bin/bash
# Same-box A/B on config 2 (tools/sweep_routes.py, auto route, 2 / 3 row chains): k_gl4t N = 192
# layers on 192- vs 96-column workgroups (SKELDIFF_GL4T_CT3), alternated twice.
OUT=gpurun_out/ab4_r03
mkdir -p $OUT
for i in 1 2; do
  for E in "SKELDIFF_GL4T_CT3=0" "SKELDIFF_GL4T_CT3=1"; do
    env $E SWEEP_ROUTES=0 SWEEP_CHAINS=2,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16 > $OUT/s.log 2>&1
    rc=$?; echo "$E rc=$rc: $(grep '^{' $OUT/s.log | python3 -c "import json,sys; print(' '.join(f\"c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  done
done
