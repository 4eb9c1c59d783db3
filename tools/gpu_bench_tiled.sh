#!/bin/bash
# bench lines: one-kernel default, tiled 1 chain, tiled 3 chains with k_gl4t holding its CU
OUT=gpurun_out/btiled
mkdir -p $OUT
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps ${STEPS:-3} --warmup 1"
run() {  # name, env, args
  env $2 timeout -k 10 300 python bench.py $B $3 > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed: $1"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$1', round(d['value']), round(d['ms_per_step'],1))"
}
run "one-kernel 3 chains" "X=1" ""
run "tiled 1 chain" "X=1" "--option split_route=3 --option row_chains=1"
run "tiled 3 chains, k_gl4t CU-exclusive" "SKELDIFF_DIAG=128" "--option split_route=3 --option row_chains=3"
run "tiled 2 chains, k_gl4t CU-exclusive" "SKELDIFF_DIAG=128" "--option split_route=3 --option row_chains=2"
