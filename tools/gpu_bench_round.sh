#!/bin/bash
# One GPU session: targeted tests, the bench line, strong-scaling per-rank proxies, config 4,
# and a rocprofv3 kernel-trace summary of the bench command.  Output under gpurun_out/$TAG/.
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
  echo "pytest rc=$?"
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
echo "bench ok"
for b in 32 16 8; do
  timeout -k 10 300 python bench.py --batch $b --no-cpu-baseline --no-exact-line --profile-reps 2 > $OUT/bench_b$b.json 2>> $OUT/bench.err || exit 1
done
timeout -k 10 300 python bench.py --config h36m_t1000 --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 2 > $OUT/bench_cfg4.json 2>> $OUT/bench.err || exit 1
echo "proxies ok"
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof.log 2>&1
  echo "rocprof rc=$?"
fi
