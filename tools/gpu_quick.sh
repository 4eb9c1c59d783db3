#!/bin/bash
# GPU test suite + default bench line + the small-batch A/B (tools/gpu_small.sh).
# usage: bash tools/gpu_quick.sh <tag>
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']), round(d['ms_per_step'],1), d['config']['route'], d['config']['row_chains'], round(d['roofline']['frac'],3), d['cpu_baseline']['value'], d['cpu_baseline']['cores'])")"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_small.sh ${TAG}_small
