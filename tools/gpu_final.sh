#!/bin/bash
# the round-end sequence on the committed binary: GPU tests, smoke(), default bench line
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $OUT/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), d['cpu_baseline']['value'])")"
