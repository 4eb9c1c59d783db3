#!/bin/bash
# J = 51 (config 3): v5 GEMM phase on k_gl4t vs k_gl4y (SKELDIFF_DIAG=1024), 1 vs 3 row chains;
# MANO T=10 golden parity; rocprofv3 kernel stats of the k_gl4t run
OUT=gpurun_out/j51
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mano or v5" tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--config mano51 --no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
run() {
  env $2 timeout -k 10 300 python bench.py $B $3 > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed: $1"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$1', round(d['value']), round(d['ms_per_step'],1))"
}
run "k_gl4y 3 chains" "SKELDIFF_DIAG=1024" ""
run "k_gl4t 3 chains (CU-exclusive)" "X=1" ""
run "k_gl4t 1 chain" "X=1" "--option row_chains=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 --option row_chains=1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
