#!/bin/bash
# DESIGN.md §4c, round 3 (second run): the update kernel's self-check + workgroup co-residency log
# on the CU-sharing diagnostic build (tools/hazard_snap.py with SKELDIFF_DIAG bit 15)
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_share.so SKELDIFF_DIAG=32768 timeout -k 10 300 \
    python -u tools/hazard_snap.py 3 2 > $OUT/selfcheck.log 2>&1
echo "rc=$?"
