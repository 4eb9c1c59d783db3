#!/bin/bash
# MODE 3 at J = 21 without the whole-CU reservation on one chain: bitwise tests + A/B vs DIAG-free
OUT=gpurun_out/j21b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
for i in 1 2; do
  for cfg in amass21 freeman17 amass16; do
    timeout -k 10 300 python bench.py --config $cfg $B > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg', round(d['value'],1), round(d['ms_per_step'],1))"
  done
done
