#!/bin/bash
# rocprofv3 kernel stats (csv) of one bench config: top kernels by total time
TAG=${TAG:-kprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config ${CFG:-amass16} --steps 1 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
for line in open(out + "/prof.log"):
    if line.startswith("{"):
        d = json.loads(line); print("bench", round(d["value"], 1), round(d["ms_per_step"], 2))
f = glob.glob(out + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), round(float(r["Percentage"]), 1))
PY
