#!/bin/bash
# GPU test suite + default bench line + rocprofv3 profile of the bench (tools/prof_bench.sh).
# usage: bash tools/gpu_session.sh <tag> [extra config for a second profile, e.g. mano51]
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']), round(d['ms_per_step'],1), d['config']['route'], d['config']['row_chains'], round(d['roofline']['frac'],3), d['cpu_baseline']['value'], d['cpu_baseline']['cores'])")"
[ $rc -eq 0 ] || exit $rc
bash tools/prof_bench.sh $TAG || exit $?
if [ -n "$2" ]; then
  timeout -k 10 600 python -u bench.py --config $2 --no-cpu-baseline --no-exact-line > $OUT/bench_$2.json 2> $OUT/bench_$2.err
  rc=$?; echo "bench $2 rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$2.json'));print(round(d['value']), round(d['ms_per_step'],1), d['config']['route'])")"
  [ $rc -eq 0 ] || exit $rc
  bash tools/prof_bench.sh ${TAG}_$2 --config $2
fi
