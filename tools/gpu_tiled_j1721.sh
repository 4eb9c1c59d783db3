#!/bin/bash
# J = 17 / 21 at the config-2 shape: one-kernel route (3 chains) vs the tiled split route (1 chain)
OUT=gpurun_out/t1721
mkdir -p $OUT
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for cfg in amass21 freeman17; do
  for opts in "" "--option split_route=3 --option row_chains=1" "--option split_route=3 --option row_chains=3"; do
    timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value']), round(d['ms_per_step'],1))"
  done
done
