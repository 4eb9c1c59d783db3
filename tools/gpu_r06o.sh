#!/bin/bash
# round 6: row-chain start stagger (SKELDIFF_CHAIN_STAGGER, µs per chain index) on config 2, same box
set -o pipefail
OUT=gpurun_out/${1:-r06o}
mkdir -p $OUT
b() {  # name, stagger, args
  local name=$1 st=$2; shift 2
  SKELDIFF_CHAIN_STAGGER=$st timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
for rep in 1 2; do
  for st in 0 15 30 60 640; do
    b st${st}_$rep $st || exit $?
  done
done
