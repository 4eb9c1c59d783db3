#!/bin/bash
# round 6: strong-scaling shard proxies (400 / 800 rows = one rank of config 2 over 8 / 4 GPUs) on
# 1, 2 and 3 row chains (auto is 2 at 129-1,200 rows)
set -o pipefail
OUT=gpurun_out/${1:-r06k}
mkdir -p $OUT
b() {  # name, args
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2), d['config'].get('row_chains'))")"
}
for rows in 8 16; do
  for c in 1 2 3; do
    b b${rows}_c$c --batch $rows --option row_chains=$c || exit $?
  done
  b b${rows}_auto --batch $rows || exit $?
done
