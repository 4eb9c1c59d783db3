#!/bin/bash
# round-4 check after the ISA audit fixes: GPU tests, config 2 / MANO / config 5 bench lines, and a
# kernel-trace of the MANO bench (per-kernel averages).
set -o pipefail
OUT=gpurun_out/${1:-r04t}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
for C in amass16 mano51 freeman17_bf16 h36m_t1000; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-exact-line > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print(round(d['value'],1), round(d['ms_per_step'],2), d['config'].get('route'))")"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mano -o run -- \
    python3 bench.py --config mano51 --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof_mano.log 2>&1
rc=$?; echo "prof mano rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"
