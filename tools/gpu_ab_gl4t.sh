#!/bin/bash
# k_gl4t K-loop form A/B on one box: SKELDIFF_GL4T_CFG values given as arguments
# (5 round-3 register-staged weights, 6 LDS-DMA ring, 7 ring + product-major MFMA order), full
# batches at J = 16 / 17 / 21, 1 and 3 row chains, each form twice, interleaved.
# usage: bash tools/gpu_ab_gl4t.sh <tag> <cfg> <cfg> ...
TAG=${1:-ab_gl4t}
shift
CFGS=${*:-6 5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
for cfg in $CFGS; do
  SKELDIFF_GL4T_CFG=$cfg SWEEP_ROUTES=0 SWEEP_CHAINS=1,3 timeout -k 10 300 python -u tools/sweep_routes.py ${CONFIGS:-amass16 freeman17 amass21} \
      >> $OUT/sweep_cfg$cfg.txt 2>> $OUT/sweep_cfg$cfg.err
  rc=$?; echo "cfg $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $OUT/sweep_cfg$cfg.txt | tail -6 | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['config'], d['row_chains'], round(d['futures_per_s']))"
done
done
