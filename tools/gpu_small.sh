#!/bin/bash
# Small-batch A/B on one GPU (DESIGN.md §4d'): config 4 (50 rows, T = 1000) and the 400 / 800-row
# strong-scaling shards of config 2 under split_route 2 (k_gl4y + MODE 2 / 3) vs the default
# (auto: the fused small-batch tile k_gl4 MODE 4 for the plain graph-linears), then a rocprofv3
# kernel trace of config 4 and its per-step gap summary (tools/trace_gaps.py).
# usage: bash tools/gpu_small.sh <tag>
TAG=${1:-small}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for spec in "h36m_t1000" "amass16 --batch 8" "amass16 --batch 16"; do
  for opt in "--option split_route=2" ""; do
    name=$(echo "$spec $opt" | tr ' =' '__')
    timeout -k 10 300 python -u bench.py --config $spec --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line $opt \
        > $OUT/bench_$name.json 2> $OUT/bench_$name.err
    rc=$?; echo "$spec $opt rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(round(d['value'],1), round(d['ms_per_step'],2), d['config'].get('route'))" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --config h36m_t1000 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 \
    > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_gaps.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) --steps 20 > $OUT/gaps.txt 2>&1
echo "gaps rc=$?"; head -12 $OUT/gaps.txt
