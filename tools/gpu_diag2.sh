#!/bin/bash
# Localise the concurrent-chain mismatch of the tiled split route: which chain's rows, at T = 1 / 2 / 4
OUT=gpurun_out/diag2
mkdir -p $OUT
for T in 1 2 4; do
  SKELDIFF_DIAG=${DIAG:-0} TILED_RUNS="one-kernel,tiled 3 chains,tiled 2 chains" timeout -k 10 200 python -u tools/tiled_check.py amass16 $T 64 > $OUT/check_T$T.log 2>&1
  rc=$?; echo "== T=$T rc=$rc"; grep -v amdgpu.ids $OUT/check_T$T.log
  [ $rc -le 1 ] || exit 1
done
