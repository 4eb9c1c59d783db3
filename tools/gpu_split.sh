#!/bin/bash
# Split route: bitwise tests, then per-batch throughput with the route forced off
# (SKELDIFF_SPLIT_ROWS=0) and on (large threshold).  Output under gpurun_out/$TAG/.
TAG=${TAG:-split}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  echo "pytest rc=$?"
  tail -3 $OUT/pytest.log
fi
for b in ${BATCHES:-8 16 32}; do
  for sr in 0 100000; do
    SKELDIFF_SPLIT_ROWS=$sr timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/b${b}_s${sr}.json 2>> $OUT/bench.err || exit 1
    echo "b=$b split_rows=$sr $(python -c "import json;d=json.load(open('$OUT/b${b}_s${sr}.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for sr in 0 100000; do
  SKELDIFF_SPLIT_ROWS=$sr timeout -k 10 300 python bench.py --config h36m_t1000 --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/cfg4_s${sr}.json 2>> $OUT/bench.err || exit 1
  echo "cfg4 split_rows=$sr $(python -c "import json;d=json.load(open('$OUT/cfg4_s${sr}.json'));print(d['value'], d['ms_per_step'])")"
done
