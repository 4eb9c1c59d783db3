#!/bin/bash
# Round-2 session: full GPU suite on the library with the tiled route auto for J = 17 / 21, then
# the affected configs (auto route vs the one-kernel route)
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for run in "amass21|" "amass21|--option split_route=1" "freeman17|" "freeman17|--option split_route=1" \
           "freeman17_half|" "freeman17_half|--option split_route=3 --option row_chains=1" "amass16|"; do
  cfg=${run%%|*}; opts=${run#*|}
  timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed $run"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value']), round(d['ms_per_step'],1))"
done
