#!/bin/bash
# Same-box A/B of bench lines (MI355X boxes differ by up to ~6 %, so route and kernel decisions
# compare runs of ONE gpurun call).  Each argument is "<config>|<bench options>"; every argument
# runs REPS times, interleaved.  Example (the config-2 route decision, DESIGN.md §4f'):
#   gpurun -- 'bash tools/gpu_ab.sh "amass16|" "amass16|--option split_route=1"'
# Environment: REPS (default 2), STEPS (default 3), ENVS (space-separated VAR=value applied to all).
OUT=gpurun_out/ab
mkdir -p $OUT
B="--no-cpu-baseline --no-exact-line --profile-reps 1 --steps ${STEPS:-3} --warmup 1"
for i in $(seq ${REPS:-2}); do
  for run in "$@"; do
    cfg=${run%%|*}; opts=${run#*|}
    env ${ENVS:-X=1} timeout -k 10 300 python bench.py --config $cfg $B $opts > $OUT/b.json 2>> $OUT/b.err || { echo "bench failed: $run"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg [$opts]', round(d['value'],1), 'futures/s', round(d['ms_per_step'],1), 'ms/step', 'update', round(d['update_kernel']['avg_launch_ms']*1e3,1), 'us')"
  done
done
