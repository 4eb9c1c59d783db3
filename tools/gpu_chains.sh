#!/bin/bash
# row-chain count sweep of the config-2 bench line (bench.py --option row_chains=N), two passes
OUT=gpurun_out/${1:-chains}
mkdir -p $OUT
for rep in 1 2; do
for n in 2 3 4 6 8; do
  timeout -k 10 200 python -u bench.py --option row_chains=$n --no-cpu-baseline --no-exact-line > $OUT/bench_c$n.$rep.json 2> $OUT/bench_c$n.$rep.err
  rc=$?; echo "chains $n rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_c$n.$rep.json'));print(round(d['value']), round(d['ms_per_step'],2), d['config'].get('row_chains'))")"
  [ $rc -eq 0 ] || exit $rc
done
done
