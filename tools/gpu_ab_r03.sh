#!/bin/bash
# Round-3 same-box A/B (one gpurun call): the posterior-update forms (bitwise test + config-2 line),
# the k_gl4t K = 192 forms (SKELDIFF_GL4T_CFG) x split route 3 (tiled everywhere) / 4 (tiled GEMM
# phase, fused one-kernel attention) x 1 / 3 row chains on config 2, and the small-batch chain
# counts (config 4 at 50 rows, the 400-row strong-scaling shard).
# usage: bash tools/gpu_ab_r03.sh [tag]
OUT=gpurun_out/${1:-ab_r03}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_v5.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_upd.log 2>&1
rc=$?; echo "update + v5 mix tests rc=$rc: $(tail -1 $OUT/pytest_upd.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mano or v5" > $OUT/pytest_v5.log 2>&1
rc=$?; echo "mano / v5 tests rc=$rc: $(tail -1 $OUT/pytest_v5.log)"; [ $rc -eq 0 ] || exit $rc
for U in 1 0; do
  SKELDIFF_UPDATE_KERNEL=$U timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-line > $OUT/bench_u$U.json 2> $OUT/bench_u$U.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench U=$U rc=$rc"; exit $rc; }
  echo "update kernel $U: $(python3 -c "import json;d=json.load(open('$OUT/bench_u$U.json'));u=d['update_kernel'];print(round(d['value']), 'futures/s; update', round(u['avg_launch_ms']*1e3,1), 'us', round(u['achieved']), 'GB/s')")"
done
for CFG in ${CFGS:-0 2 3 4}; do
  SKELDIFF_GL4T_CFG=$CFG SWEEP_ROUTES=3,4 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py amass16 > $OUT/sweep_gl4t$CFG.log 2>&1
  rc=$?; echo "GL4T_CFG $CFG rc=$rc: $(grep '^{' $OUT/sweep_gl4t$CFG.log | python3 -c "import json,sys; print(' '.join(f\"r{r['split_route']}c{r['row_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"
  [ $rc -eq 0 ] || exit $rc
done
for M in 1 0; do
  SKELDIFF_V5_MIX=$M SWEEP_ROUTES=0 SWEEP_CHAINS=1 timeout -k 10 300 python -u tools/sweep_routes.py mano51 > $OUT/sweep_v5mix$M.log 2>&1
  rc=$?; echo "V5_MIX $M rc=$rc: $(grep '^{' $OUT/sweep_v5mix$M.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"
  [ $rc -eq 0 ] || exit $rc
done
for PF in 12 8; do
  SKELDIFF_GL4Y_PF=$PF SWEEP_ROUTES=0 SWEEP_CHAINS=1,2,3 timeout -k 10 300 python -u tools/sweep_routes.py h36m_t1000 amass16:8 amass16:16 > $OUT/sweep_small_pf$PF.log 2>&1
  rc=$?; echo "small PF $PF rc=$rc: $(grep '^{' $OUT/sweep_small_pf$PF.log | python3 -c "import json,sys; print(' '.join(f\"{r['config']}/c{r['ran_chains']}={r['futures_per_s']:.0f}\" for r in map(json.loads, sys.stdin)))")"
  [ $rc -eq 0 ] || exit $rc
done
