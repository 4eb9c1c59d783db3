#!/bin/bash
# DESIGN.md §4c, round 3 (third run): first divergence with the plain update kernel, without
# LDS tables (SKELDIFF_DIAG bit 5) and holding its CU (bit 6), CU-sharing diagnostic build
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_share.so
for v in 0 32 64; do
    SKELDIFF_DIAG=$v timeout -k 10 300 python -u tools/hazard_snap.py 3 2 > $OUT/snap_d$v.log 2>&1
    rc=$?
    echo "diag $v rc=$rc: $(grep 'final latents' $OUT/snap_d$v.log)"
    [ $rc -eq 0 ] || exit 1
done
