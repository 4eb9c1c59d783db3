#!/bin/bash
# multi-unit k_gl4t (SKELDIFF_GL4T_CFG 11 / 12) on one box: the bitwise route / row-chain tests
# under each form, then the A/B against the default (8).
set -o pipefail
OUT=gpurun_out/${1:-nu}
mkdir -p $OUT
for cfg in 12 11; do
  SKELDIFF_GL4T_CFG=$cfg timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_configs.py -k "row_chains or split_route or config2 or two_" > $OUT/pytest_cfg$cfg.txt 2>&1
  rc=$?; tail -3 $OUT/pytest_cfg$cfg.txt; [ $rc -eq 0 ] || exit $rc
done
CONFIGS="amass16 freeman17" bash tools/gpu_ab_gl4t.sh ${1:-nu} 8 12 11
