#!/bin/bash
# Concurrency hazard discrimination: the tiled split route with 3 row chains,
# bitwise vs the one-kernel route, under SKELDIFF_DIAG = 0 (plain), 4 (chains serialised on one
# stream), 1 (agent release after phase 1), 2 (agent acquire before phase 2), 3 (both).
OUT=gpurun_out/diag
mkdir -p $OUT
for d in ${DIAGS:-0 4 1 2 3}; do
  SKELDIFF_DIAG=$d timeout -k 10 200 python -u tools/tiled_check.py amass16 4 64 > $OUT/check_$d.log 2>&1
  rc=$?; echo "== DIAG=$d rc=$rc"; grep -v amdgpu.ids $OUT/check_$d.log
  [ $rc -le 1 ] || exit 1
done
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
timeout -k 10 300 python bench.py $B --option split_route=3 --option row_chains=1 > $OUT/bench.json 2>> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('tiled 1 chain', round(d['value']), round(d['ms_per_step'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 --option split_route=3 --option row_chains=1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
