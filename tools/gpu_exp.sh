#!/bin/bash
# v4 timing experiments (SKELDIFF_GL4_CFG 0 full / 1 loads only / 2 no epilogue / 3 no split VALU)
mkdir -p gpurun_out
for rows in ${ROWSET:-3200 12800}; do
for cfg in ${CFGS:-0 1 2 3}; do
  ROWS=$rows SKELDIFF_GL_VARIANT=4 SKELDIFF_GL4_CFG=$cfg timeout -k 10 120 python -u tools/bench_gl.py > gpurun_out/exp_${rows}_${cfg}.log 2>&1 || exit $?
  echo "rows=$rows cfg=$cfg"; grep -v amdgpu gpurun_out/exp_${rows}_${cfg}.log | grep -E "res_block1|to_qkv|per-step"
done
done
