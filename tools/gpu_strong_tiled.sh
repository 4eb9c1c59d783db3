#!/bin/bash
# strong-scaling per-rank proxies (64 sequences over 2 / 4 / 8 ranks) and config 4: default route
# vs the tiled split route on one chain
OUT=gpurun_out/strong
mkdir -p $OUT
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for b in 32 16 8; do
  for opts in "" "--option split_route=3 --option row_chains=1"; do
    timeout -k 10 300 python bench.py --batch $b $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('batch $b [$opts]', round(d['value']), round(d['ms_per_step'],1))"
  done
done
