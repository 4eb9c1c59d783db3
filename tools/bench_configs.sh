#!/bin/bash
# One bench line per BASELINE config shape (1 GPU) + the strong-scaling per-rank shards of config 2
# (32 / 16 / 8 sequences = 1,600 / 800 / 400 rows: one rank of 2 / 4 / 8 GPUs), for DESIGN.md.
# usage: bash tools/bench_configs.sh [out dir under gpurun_out]
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; return $rc; }
  python3 -c "import json; r=json.load(open('$OUT/$name.json')); print('$name |', r['config']['rows_per_gpu'], 'rows | T', r['config']['T'], '|', round(r['value'],1), r['unit'], '|', r['config']['route'], '| chains', r['config']['row_chains'], '| timed frac', round(r['roofline']['timed_region']['frac'],3))"
}
for cfg in ${CFGS:-amass16 amass21 freeman17 freeman17_half freeman17_bf16 mano51 mano52 h36m_t1000}; do
  run cfg_$cfg --config $cfg || exit $?
done
for b in 32 16 8; do
  run strong_b$b --config amass16 --batch $b || exit $?
done
