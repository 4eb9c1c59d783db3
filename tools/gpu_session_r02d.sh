#!/bin/bash
# tiled route for half precision (J = 17 auto; J = 16 half: tiled vs one-kernel) + parity subset
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_precision.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for run in "freeman17_half|" "amass16|--precision half" "amass16|--precision half --option split_route=3 --option row_chains=1" \
           "amass21|--precision half" "amass21|--precision half --option split_route=1"; do
  cfg=${run%%|*}; opts=${run#*|}
  timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed $run"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value']), round(d['ms_per_step'],1))"
done
