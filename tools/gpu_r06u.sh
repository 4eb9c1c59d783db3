#!/bin/bash
# round 6: 2 vs 3 row chains at the strong-scaling shard sizes (400 / 600 rows), 3 reps, same box
set -o pipefail
OUT=gpurun_out/${1:-r06u}
mkdir -p $OUT
b() {  # name, args
  local name=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
for rep in ${REPS:-1 2 3}; do
  for seq in ${SEQS:-8 12}; do
    b s${seq}_c1_$rep --batch $seq --option row_chains=1 && b s${seq}_c2_$rep --batch $seq --option row_chains=2 && b s${seq}_c3_$rep --batch $seq --option row_chains=3 || exit $?
  done
done
