#!/bin/bash
# round 6: register-x library vs the round-5 ring (libskeldiff_prev.so) at 1 and 2 row chains, config 2
set -o pipefail
OUT=gpurun_out/${1:-r06n}
mkdir -p $OUT
PREV=$PWD/skeletondiffusion_amd/libskeldiff_prev.so
b() {  # name, lib, args
  local name=$1 lib=$2; shift 2
  SKELDIFF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
NEW=$PWD/skeletondiffusion_amd/libskeldiff.so
for c in 1 2 3; do
  b new_c$c $NEW --option row_chains=$c && b old_c$c $PREV --option row_chains=$c || exit $?
done
