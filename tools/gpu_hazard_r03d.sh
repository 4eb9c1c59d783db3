#!/bin/bash
# DESIGN.md §4c, round 3 (fourth run): placement and visibility discriminators on the CU-sharing
# diagnostic build, tools/tiled_check.py (config 2, T = 4, one-kernel route vs three tiled chains)
#   8192          chains on contiguous CU-index ranges (disjoint CUs)
#   8192+131072   chains on interleaved CU indices (cu % 3): disjoint CUs, every chain on every XCD
#   65536         every wave of the v4 / update kernels ends with an agent-scope release
#   65536+8       release at every end + agent-scope acquire at every start
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_share.so TILED_RUNS="one-kernel,tiled 3 chains"
for v in 0 8192 139264 65536 65544 0; do
    SKELDIFF_DIAG=$v timeout -k 10 200 python -u tools/tiled_check.py amass16 4 64 > $OUT/d_$v.log 2>&1
    rc=$?
    echo "diag $v rc=$rc: $(grep 'tiled 3 chains' $OUT/d_$v.log | sed 's/first rows.*//' | tr '\n' ' ')"
    [ $rc -le 1 ] || exit 1
done
