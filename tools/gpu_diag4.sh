#!/bin/bash
# Concurrent-chain mismatch: which co-residency triggers it?  SKELDIFF_DIAG 32 = the
# update kernel without LDS, 64 = it holds its CU, 128 = k_gl4t holds its CU, 256 = MODE 2 holds its CU
OUT=gpurun_out/diag4
mkdir -p $OUT
for d in ${DIAGS:-512}; do
  for T in ${TS:-4}; do
    SKELDIFF_DIAG=$d TILED_RUNS="one-kernel,tiled 3 chains,tiled 2 chains" timeout -k 10 200 python -u tools/tiled_check.py amass16 $T 64 > $OUT/check_${d}_$T.log 2>&1
    rc=$?; echo "== DIAG=$d T=$T rc=$rc"; grep -v amdgpu.ids $OUT/check_${d}_$T.log
    [ $rc -le 1 ] || exit 1
  done
done
