#!/bin/bash
# Tiled split route (k_gl4t) session: optional full GPU suite, bitwise check vs the one-kernel
# route at the config-2 shape, bench lines per route / chain count, rocprofv3 kernel stats.
TAG=${TAG:-tiled}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$SUITE" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python -u tools/tiled_check.py amass16 4 64 > $OUT/check.log 2>&1
rc=$?; cat $OUT/check.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps ${STEPS:-3} --warmup 1"
for opts in "" "--option split_route=3 --option row_chains=1" "--option split_route=3 --option row_chains=3" ${EXTRA_RUNS}; do
  timeout -k 10 300 python bench.py $B $opts > $OUT/bench.json 2>> $OUT/bench.err || { echo "bench failed: $opts"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/bench.json'));print('bench [$opts]', round(d['value']), round(d['ms_per_step'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 --option split_route=3 --option row_chains=1 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
python3 - $OUT <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(out + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
