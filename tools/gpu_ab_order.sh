#!/bin/bash
# k_gl4t work order: node-major (default) vs row-group-major (SKELDIFF_DIAG=4096), same box;
# tiled-route bitwise tests first
OUT=gpurun_out/ab_order
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "tiled or config2 or split" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps 5 --warmup 2"
for i in 1 2; do
  for d in 0 4096; do
    for cfg in amass16 freeman17; do
      SKELDIFF_DIAG=$d timeout -k 10 300 python bench.py --config $cfg $B > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed"; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg DIAG=$d', round(d['value'],1), round(d['ms_per_step'],1))"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $B --steps 1 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), round(float(r["Percentage"]), 1))
PY
