#!/bin/bash
# round 6: register-x k_gl4t -- GPU suite + smoke + bench, then a same-box A/B of the bench
# (default config 2 and config 3) against the previous library (skeletondiffusion_amd/libskeldiff_prev.so)
set -o pipefail
TAG=${1:-r06g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_final.sh $TAG || exit $?
PREV=$PWD/skeletondiffusion_amd/libskeldiff_prev.so
for rep in 1 2; do
  for cfg in amass16 mano51; do
    timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline --no-exact-line > $OUT/new_${cfg}_$rep.json 2> $OUT/new_${cfg}_$rep.err || exit $?
    SKELDIFF_LIB=$PREV timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline --no-exact-line > $OUT/old_${cfg}_$rep.json 2> $OUT/old_${cfg}_$rep.err || exit $?
    echo "$cfg rep $rep new $(python3 -c "import json;print(round(json.load(open('$OUT/new_${cfg}_$rep.json'))['value'],1))") old $(python3 -c "import json;print(round(json.load(open('$OUT/old_${cfg}_$rep.json'))['value'],1))")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/trace.log 2>&1
echo "trace rc=$?"
