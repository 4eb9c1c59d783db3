#!/bin/bash
# J = 51: k_gl5_mix with J-sized LDS, k_update1 vs the pair form (SKELDIFF_DIAG=2048); parity subset
OUT=gpurun_out/j51b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mano or v5 or single_step" tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--config mano51 --no-cpu-baseline --no-exact-line --profile-reps 1 --steps 2 --warmup 1"
for d in 2048 0; do
  SKELDIFF_DIAG=$d timeout -k 10 300 python bench.py $B > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('DIAG=$d', round(d['value']), round(d['ms_per_step'],1), d['update_kernel'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
