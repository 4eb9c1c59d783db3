#!/bin/bash
# the row-chain hazard on the CU-sharing diagnostic build
# (libskeldiff_share.so: k_gl4t shares CUs under three row chains).
#   base   -- reproduction (tools/tiled_check.py, T = 4, config 2)
#   cumask -- the chains on disjoint CU sets (SKELDIFF_DIAG bit 13)
#   args   -- every workgroup re-hashes its argument block (bit 14; status bits 0x100..0x800)
#   snap   -- first divergent (step, call) between one and three chains (tools/hazard_snap.py)
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_share.so TILED_RUNS="one-kernel,tiled 3 chains"
run() {  # name diag cmd...
    local name=$1 diag=$2
    shift 2
    SKELDIFF_DIAG=$diag timeout -k 10 240 "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc: $(grep -v amdgpu.ids $OUT/$name.log | tail -1)"
    [ $rc -le 1 ]
}
run base 0 python -u tools/tiled_check.py amass16 4 64 &&
run cumask 8192 python -u tools/tiled_check.py amass16 4 64 &&
run args 16384 python -u tools/tiled_check.py amass16 4 64 &&
run snap 0 python -u tools/hazard_snap.py 3 2
