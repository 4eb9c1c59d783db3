#!/bin/bash
# Throughput sweep over batch x row chains x split route (SKELDIFF_* process defaults)
TAG=${TAG:-sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for b in ${BATCHES:-8 16 32}; do
  for ch in ${CHAINS:-1 3}; do
    for sr in ${SPLITS:-0 100000}; do
      SKELDIFF_CHAINS=$ch SKELDIFF_SPLIT_ROWS=$sr timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/b${b}_c${ch}_s${sr}.json 2>> $OUT/bench.err || exit 1
      echo "b=$b chains=$ch split_rows=$sr $(python -c "import json;d=json.load(open('$OUT/b${b}_c${ch}_s${sr}.json'));print(round(d['value']), round(d['ms_per_step'],2))")"
    done
  done
done
