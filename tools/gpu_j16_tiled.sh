#!/bin/bash
# J = 16 after the MODE 3 LDS change: one-kernel (3 chains) vs tiled split route (1 chain), f32 and half
OUT=gpurun_out/j16t
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
for run in "|" "|--option split_route=3 --option row_chains=1" "|--precision half" "|--precision half --option split_route=3 --option row_chains=1" "|" "|--option split_route=3 --option row_chains=1"; do
  opts=${run#*|}
  timeout -k 10 300 python bench.py $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed $run"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('amass16 [$opts]', round(d['value'],1), round(d['ms_per_step'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 --option split_route=3 --option row_chains=1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
