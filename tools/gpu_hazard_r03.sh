#!/bin/bash
# DESIGN.md §4c (round 3): the experiments that localised the row-chain hazard, one mode per GPU
# call; logs in gpurun_out/hazard_r03 (copies under profiles/r03_hazard).  They need a library
# built WITH packed-FP32 code and k_gl4t sharing CUs (the round-2 state), e.g.
#   build_library(extra=[...], tag="_share", packed_fp32=True)  -> libskeldiff_share.so
# (the product library, without packed FP32, is exact in every mode).
#   base      reproduction: tools/tiled_check.py, config 2, T = 4, one-kernel vs three tiled chains
#   placement SKELDIFF_DIAG 8192: chains on disjoint contiguous CU ranges; 139264: interleaved
#   snap      tools/hazard_snap.py: first divergent (step, call) between one and three chains
#   dump      the same with the first update's inputs dumped (HAZARD_DUMP=1)
#   nopk      LIB2 (built without packed FP32) vs LIB, x3 (tiled_check)
MODE=${1:-base}
LIB=${LIB:-skeletondiffusion_amd/libskeldiff_share.so}
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export TILED_RUNS="one-kernel,tiled 3 chains"
check() {  # name diag lib
    SKELDIFF_LIB=$3 SKELDIFF_DIAG=$2 timeout -k 10 240 python -u tools/tiled_check.py amass16 4 64 > $OUT/$1.log 2>&1
    local rc=$?
    echo "$1 rc=$rc: $(grep 'tiled 3 chains' $OUT/$1.log | sed 's/first rows.*//' | tr '\n' ' ')"
    [ $rc -le 1 ]
}
case $MODE in
  base) check base 0 $LIB ;;
  placement) check d_8192 8192 $LIB && check d_139264 139264 $LIB ;;
  snap) SKELDIFF_LIB=$LIB timeout -k 10 400 python -u tools/hazard_snap.py 3 2 > $OUT/snap.log 2>&1; echo "rc=$?" ;;
  dump) SKELDIFF_LIB=$LIB HAZARD_DUMP=1 timeout -k 10 400 python -u tools/hazard_snap.py 3 2 > $OUT/dump.log 2>&1; echo "rc=$?" ;;
  nopk) for i in 1 2 3; do check nopk_$i 0 ${LIB2:-skeletondiffusion_amd/libskeldiff_nopk.so} || exit 1; done; check pk 0 $LIB ;;
esac
