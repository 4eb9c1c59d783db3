#!/bin/bash
# Same-box repeat of the mid-batch / small-batch chain sweeps (tools/sweep_routes.py), twice.
OUT=gpurun_out/ab3_r03
mkdir -p $OUT
for i in 1 2; do
  SWEEP_ROUTES=0,1 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16:16 > $OUT/mid$i.log 2>&1
  rc=$?; echo "mid$i rc=$rc: $(grep '^{' $OUT/mid$i.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}/r{r['split_route']}c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
  SWEEP_ROUTES=0 SWEEP_CHAINS=1,2 timeout -k 10 300 python -u tools/sweep_routes.py h36m_t1000 > $OUT/c4_$i.log 2>&1
  rc=$?; echo "c4_$i rc=$rc: $(grep '^{' $OUT/c4_$i.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}/r{r['split_route']}c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"; [ $rc -eq 0 ] || exit $rc
done
