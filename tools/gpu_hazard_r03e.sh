#!/bin/bash
# DESIGN.md §4c, round 3 (fifth run): provenance of the update kernel's wrong inputs
# (tools/hazard_snap.py with HAZARD_DUMP=1, CU-sharing diagnostic build); twice
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_share.so HAZARD_DUMP=1
for i in 1 2; do
    timeout -k 10 400 python -u tools/hazard_snap.py 3 2 > $OUT/dump_$i.log 2>&1
    rc=$?
    echo "run $i rc=$rc: $(grep 'final latents' $OUT/dump_$i.log)"
    [ $rc -eq 0 ] || exit 1
done
