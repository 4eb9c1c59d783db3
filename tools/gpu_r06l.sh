#!/bin/bash
# round 6: same-box A/B of plan options on config 2 (default vs fused one-kernel attention tile
# for to_qkv = split_route 4, update_kernel 1)
set -o pipefail
OUT=gpurun_out/${1:-r06l}
mkdir -p $OUT
b() {  # name, args
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
for rep in 1 2; do
  b def_$rep && b r4_$rep --option split_route=4 && b upd1_$rep --option update_kernel=1 || exit $?
done
