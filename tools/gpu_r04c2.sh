#!/bin/bash
# config-2 check: all GPU tests, two default bench lines and a kernel trace of the bench
set -o pipefail
OUT=gpurun_out/${1:-r04c2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py > $OUT/bench.$rep.json 2> $OUT/bench.$rep.err
  rc=$?; echo "bench rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench.$rep.json'));print(round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3))")"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof.log 2>&1
echo "prof rc=$?"
