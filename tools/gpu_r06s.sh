#!/bin/bash
# round 6: k_gl4t chunks in flight (PF 2 product vs -DSD_GL4T_PF=3 / 4 builds) on config 2 and 3,
# same box; the bitwise route tests under each variant first
set -o pipefail
OUT=gpurun_out/${1:-r06s}
mkdir -p $OUT
for v in pf3 pf4; do
  SKELDIFF_LIB=$PWD/skeletondiffusion_amd/libskeldiff_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_configs.py -k "tiled or config2_as_benched or config3_as_benched or split_route" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
b() {  # name, lib, args
  local name=$1 lib=$2; shift 2
  SKELDIFF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
L=$PWD/skeletondiffusion_amd
for rep in 1 2; do
  b pf2_$rep $L/libskeldiff.so && b pf3_$rep $L/libskeldiff_pf3.so && b pf4_$rep $L/libskeldiff_pf4.so || exit $?
done
b b16_pf2 $L/libskeldiff.so --batch 16 && b b16_pf3 $L/libskeldiff_pf3.so --batch 16 && b b16_pf4 $L/libskeldiff_pf4.so --batch 16
