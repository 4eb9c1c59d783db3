#!/bin/bash
# Split-route check: bitwise tests + config-4 bench + rocprofv3 kernel stats (csv)
TAG=${TAG:-split}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k split -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config ${CFG:-h36m_t1000} --steps 1 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 ${BENCH_ARGS} > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
for line in open(out + "/prof.log"):
    if line.startswith("{"):
        d = json.loads(line); print("bench", d["value"], d["ms_per_step"])
f = glob.glob(out + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
