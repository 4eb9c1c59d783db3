#!/bin/bash
# DESIGN.md §4c probes: k_gl4t sharing CUs under three row chains (diagnostic builds of
# libskeldiff: _x0 = shared CUs, _x1 = + __syncthreads() at the chunk barrier, _x2 = + dynamic LDS);
# each compared bitwise with the one-kernel route by tools/tiled_check.py
OUT=gpurun_out/hazard_r02
mkdir -p $OUT
for v in x0 x1 x2; do
    SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_$v.so TILED_RUNS="one-kernel,tiled 3 chains" \
        timeout -k 10 200 python -u tools/tiled_check.py amass16 4 64 > $OUT/$v.log 2>&1
    rc=$?
    echo "$v rc=$rc: $(tail -1 $OUT/$v.log)"
    [ $rc -le 1 ] || exit 1
done
