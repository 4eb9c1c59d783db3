#!/bin/bash
# round 6: kernel traces of the register-x k_gl4t library vs the previous one (libskeldiff_prev.so)
# on config 2 / config 3, and of the strong-scaling shard sizes (400 / 800 rows)
set -o pipefail
OUT=gpurun_out/${1:-r06h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PREV=$PWD/skeletondiffusion_amd/libskeldiff_prev.so
tr() {  # name, lib, bench args
  local name=$1 lib=$2; shift 2
  SKELDIFF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line "$@" > $OUT/$name.log 2>&1
  local rc=$?; rm -f $OUT/$name/run_kernel_trace.csv  # keep the stats (gpurun_out is capped at 64 MiB)
  echo "$name rc=$rc $(grep '"metric"' $OUT/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],2))')"; return $rc
}
NEW=$PWD/skeletondiffusion_amd/libskeldiff.so
tr mano_new $NEW --config mano51 && tr mano_old $PREV --config mano51 && tr amass_old $PREV && \
tr b400_new $NEW --batch 8 && tr b800_new $NEW --batch 16 && tr b800_old $PREV --batch 16
