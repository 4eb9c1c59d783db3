#!/bin/bash
# k_update_mfma: bitwise tests vs the element-per-thread forms, then the GEMM-phase form sweep
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_upd.log 2>&1
rc=$?; echo "update tests rc=$rc: $(tail -1 $OUT/pytest_upd.log)"
[ $rc -eq 0 ] || { grep -m3 "assert\|Error" $OUT/pytest_upd.log; }
for U in 0 1; do
  SKELDIFF_UPDATE_KERNEL=$U timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-line > $OUT/bench_u$U.json 2>/dev/null
  echo "update kernel $U: $(python3 -c "import json;d=json.load(open('$OUT/bench_u$U.json'));print(round(d['value']), 'update ms', round(d['update_kernel']['avg_launch_ms']*1e3,1), 'us', round(d['update_kernel']['achieved']), 'GB/s')")"
done
TAG=r03f bash tools/gpu_gl4t_res.sh
