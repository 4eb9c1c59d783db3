#!/bin/bash
# Update / v5 / golden tests, then the MANO (config 3) and config-2 bench lines.
OUT=gpurun_out/${1:-mano}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_v5.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for C in mano51 mano52 amass16; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-exact-line > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print(round(d['value']), round(d['ms_per_step'],1), d['config']['route'], round(d['update_kernel']['avg_launch_ms']*1e3,1), 'us update')")"
  [ $rc -eq 0 ] || exit $rc
done
