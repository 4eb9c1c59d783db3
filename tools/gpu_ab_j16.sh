#!/bin/bash
# same-box A/B for config 2: auto route (tiled, one chain) vs forced one-kernel route (3 chains)
OUT=gpurun_out/ab16
mkdir -p $OUT
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 5 --warmup 2"
for i in 1 2 3; do
  for opts in "" "--option split_route=1"; do
    timeout -k 10 300 python bench.py $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('amass16 [$opts]', round(d['value'],1), round(d['ms_per_step'],1))"
  done
done
