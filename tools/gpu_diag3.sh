#!/bin/bash
# Concurrent-chain mismatch: argument/grid consistency check (SKELDIFF_DIAG bit 4 -> status 0x4)
# and the runtime's kernarg placement (HIP_FORCE_DEV_KERNARG 0 / 1)
OUT=gpurun_out/diag3
mkdir -p $OUT
for K in default 0 1; do
  if [ $K = default ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$K; fi
  SKELDIFF_DIAG=16 TILED_RUNS="one-kernel,tiled 3 chains" timeout -k 10 200 python -u tools/tiled_check.py amass16 2 64 > $OUT/check_$K.log 2>&1
  rc=$?; echo "== HIP_FORCE_DEV_KERNARG=$K rc=$rc"; grep -v amdgpu.ids $OUT/check_$K.log
  [ $rc -le 1 ] || exit 1
done
