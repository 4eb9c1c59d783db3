#!/bin/bash
# Round-end measurement session (one gpurun call): the default bench line, the rocprofv3 trace +
# PMC traffic passes of the same command (tools/profile.sh), one line per BASELINE config
# (tools/bench_configs.sh) and the strong-scaling per-rank proxies (64 sequences over 2 / 4 / 8
# ranks = 32 / 16 / 8 sequences on one GPU).  Output under gpurun_out/.
set -u
TAG=${TAG:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; exit 1; }
echo "bench ok"
bash tools/profile.sh $TAG || exit 1
CFGS=${CFGS:-"amass21 freeman17 freeman17_half freeman17_bf16 mano51 h36m_t1000"} bash tools/bench_configs.sh || exit 1
for b in 32 16 8; do
  timeout -k 10 300 python bench.py --batch $b --no-cpu-baseline --no-exact-line --profile-reps 2 > gpurun_out/$TAG/strong_b$b.json 2>> gpurun_out/$TAG/bench.err || exit 1
  echo "strong proxy b=$b $(python -c "import json;d=json.load(open('gpurun_out/$TAG/strong_b$b.json'));print(round(d['value']), round(d['ms_per_step'],2))")"
done
