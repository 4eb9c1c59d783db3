#!/bin/bash
# closing check: all GPU tests, MANO + config 2 bench lines, MANO kernel stats, training bench
set -o pipefail
OUT=gpurun_out/${1:-r04z}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
for C in mano51 amass16; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-exact-line > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mano -o run -- \
    python3 bench.py --config mano51 --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof_mano.log 2>&1
rc=$?; echo "prof mano rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_train.py --J 16 --rows 1024 --steps 10 --warmup 3 > $OUT/train16.json 2> $OUT/train16.err
echo "train rc=$?: $(python3 -c "import json;d=json.load(open('$OUT/train16.json'));print(round(d['hip']['ms_per_step'],2), round(d['torch_ops_same_gpu']['ms_per_step'],2), round(d['speedup'],2))")"
