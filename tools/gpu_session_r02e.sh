#!/bin/bash
# bf16 mode on the tiled route (k_gl4t PREC 2): bitwise vs the one-kernel route, config 5 gate, benches
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_precision.py tests/test_gpu_configs.py -k "tiled or bf16 or precision" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for run in "freeman17_bf16|" "freeman17_bf16|--option split_route=1" "freeman17_half|" "amass21|--precision bf16" "amass21|--precision bf16 --option split_route=1"; do
  cfg=${run%%|*}; opts=${run#*|}
  timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed $run"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value']), round(d['ms_per_step'],1))"
done
