#!/bin/bash
# k_gl4t K = 192 forms (SKELDIFF_GL4T_CFG 0..4, sd_graph_linear_v4.hip): bitwise tests, then a
# same-box route sweep per form
OUT=gpurun_out/${TAG:-r03e}
mkdir -p $OUT
for CFG in ${CFGS:-1 2 3 4 0}; do
  SKELDIFF_GL4T_CFG=$CFG timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tiled_split_route_bitwise or config2_as_benched" > $OUT/pytest_$CFG.log 2>&1
  rc=$?; echo "CFG $CFG pytest rc=$rc: $(tail -1 $OUT/pytest_$CFG.log)"; [ $rc -eq 0 ] || exit $rc
done
for CFG in ${CFGS:-1 2 3 4 0}; do
  SKELDIFF_GL4T_CFG=$CFG SWEEP_ROUTES=0 SWEEP_CHAINS=${CHAINS:-1,3} timeout -k 10 400 python -u tools/sweep_routes.py ${SHAPES:-amass16 freeman17 amass21} > $OUT/sweep_$CFG.log 2>&1
  echo "CFG $CFG rc=$?: $(grep '^{' $OUT/sweep_$CFG.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}/c{r['row_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"
done
