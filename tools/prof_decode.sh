cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_dec
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec -o run -- python3 tools/bench_decode.py 12800 120 > gpurun_out/prof_dec/log.txt 2>&1 || { tail -20 gpurun_out/prof_dec/log.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_dec/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:8]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", round(float(r["Percentage"]), 1), "%")
PY
