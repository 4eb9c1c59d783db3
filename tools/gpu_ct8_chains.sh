#!/bin/bash
# SKELDIFF_GL4T_CT8 x row chains on the config-2 bench line, two passes
OUT=gpurun_out/${1:-ct8ch}
mkdir -p $OUT
for rep in 1 2; do
for v in 0 1; do
for n in 2 3; do
  SKELDIFF_GL4T_CT8=$v timeout -k 10 200 python -u bench.py --option row_chains=$n --no-cpu-baseline --no-exact-line > $OUT/b_ct8${v}_c$n.$rep.json 2> $OUT/b_ct8${v}_c$n.$rep.err
  rc=$?; echo "ct8=$v chains=$n rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/b_ct8${v}_c$n.$rep.json'));print(round(d['value']))")"
  [ $rc -eq 0 ] || exit $rc
done
done
done
