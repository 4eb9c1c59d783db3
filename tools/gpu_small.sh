#!/bin/bash
# small-batch checks: GPU tests (subset), config 4 and 400 / 800 rows, update-kernel choice
TAG=${TAG:-small}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py tests/test_gpu_parity.py} -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest.log
for ur in 0 100000; do
  SKELDIFF_UPDATE_ROWS=$ur timeout -k 10 300 python bench.py --config h36m_t1000 --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/cfg4_u$ur.json 2>> $OUT/bench.err || exit 1
  echo "cfg4 update_rows=$ur $(python -c "import json;d=json.load(open('$OUT/cfg4_u$ur.json'));print(round(d['value'],1), round(d['ms_per_step'],2), d['update_kernel']['achieved'])")"
  for b in 8 16 64; do
    SKELDIFF_UPDATE_ROWS=$ur timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/b${b}_u$ur.json 2>> $OUT/bench.err || exit 1
    echo "b=$b update_rows=$ur $(python -c "import json;d=json.load(open('$OUT/b${b}_u$ur.json'));print(round(d['value']), round(d['ms_per_step'],2), d['update_kernel']['achieved'])")"
  done
done
