#!/bin/bash
# GPU tests, the training-step bench (J = 16 / 21) with its kernel trace, MANO + config 2 lines.
set -o pipefail
OUT=gpurun_out/${1:-r04u}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
for J in 16 21; do
  timeout -k 10 300 python -u tools/bench_train.py --J $J --rows 1024 --steps 10 --warmup 3 > $OUT/train$J.json 2> $OUT/train$J.err
  rc=$?; echo "train J=$J rc=$rc: $(cat $OUT/train$J.json | head -c 400)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_train -o run -- \
    python3 tools/bench_train.py --J 16 --rows 1024 --steps 3 --warmup 1 --modes hip > $OUT/prof_train.log 2>&1
rc=$?; echo "prof train rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in amass16 mano51; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-exact-line > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
  [ $rc -eq 0 ] || exit $rc
done
