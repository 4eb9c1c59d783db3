#!/bin/bash
# MODE 3 with Z aliased over the Y slab (<= 64 KB of LDS at J = 16 / 17): parity + benches
OUT=gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for run in "freeman17|" "amass21|" "freeman17_bf16|" "h36m_t1000|--steps 3" "amass16|--batch 8"; do
  cfg=${run%%|*}; opts=${run#*|}
  timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed $run"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value'],1), round(d['ms_per_step'],1))"
done
