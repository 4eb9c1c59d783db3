#!/bin/bash
# round 6: GPU suite on the library, then same-box A/B: N = 192 tile of the row-blocked k_gl4t
# (RT2 CT3, product) vs 1 x 6 (libskeldiff_ct6.so, -DSD_GL4T_RT2=0) and row-chain counts
set -o pipefail
OUT=gpurun_out/${1:-r06i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
CT6=$PWD/skeletondiffusion_amd/libskeldiff_ct6.so
b() {  # name, lib, args
  local name=$1 lib=$2; shift 2
  SKELDIFF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.json 2> $OUT/$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2))")"
}
NEW=$PWD/skeletondiffusion_amd/libskeldiff.so
for rep in 1 2; do
  b rt2_$rep $NEW && b ct6_$rep $CT6 || exit $?
done
b mano_$rep $NEW --config mano51 && \
b rt2_c2 $NEW --option row_chains=2 && b rt2_c4 $NEW --option row_chains=4 && b ct6_c4 $CT6 --option row_chains=4
