#!/bin/bash
# SKELDIFF_GL4T_CT8 A/B: the bitwise route / chain tests under CT8=1, then config 2 and MANO bench
# lines with CT8 = 0 / 1 interleaved, two passes
set -o pipefail
OUT=gpurun_out/${1:-ct8}
mkdir -p $OUT
SKELDIFF_GL4T_CT8=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_configs.py tests/test_gpu_parity.py -k "row_chains or split_route or config2 or mano or two_" > $OUT/pytest_ct8.txt 2>&1
rc=$?; echo "pytest ct8 rc=$rc: $(tail -1 $OUT/pytest_ct8.txt)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in 0 1; do
for C in amass16 mano51; do
  SKELDIFF_GL4T_CT8=$v timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-exact-line > $OUT/bench_${C}_ct8$v.$rep.json 2> $OUT/bench_${C}_ct8$v.$rep.err
  rc=$?; echo "ct8=$v $C rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_${C}_ct8$v.$rep.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
  [ $rc -eq 0 ] || exit $rc
done
done
done
