#!/bin/bash
# AMASS J = 21: kernel profile of the tiled route; one chain vs three (k_gl4t holding its CU)
OUT=gpurun_out/j21
mkdir -p $OUT
export TMPDIR=/tmp
B="--config amass21 --no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
for i in 1 2; do
  for opts in "" "--option split_route=3 --option row_chains=3"; do
    timeout -k 10 300 python bench.py $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('amass21 [$opts]', round(d['value'],1), round(d['ms_per_step'],1))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
