#!/bin/bash
# round 6: row chains {2, 3} x chain start stagger {0, 30, 45} µs on config 2, same box, 2 reps
set -o pipefail
OUT=gpurun_out/${1:-r06q}
mkdir -p $OUT
b() {  # name, stagger, args
  local name=$1 st=$2; shift 2
  SKELDIFF_CHAIN_STAGGER=$st timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
for rep in 1 2; do
  for c in 2 3; do
    for st in 0 30 45; do
      b c${c}_st${st}_$rep $st --option row_chains=$c || exit $?
    done
  done
done
