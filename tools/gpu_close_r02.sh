#!/bin/bash
# Round-2 close: smoke(), the default bench line as the driver runs it, and a rocprofv3 kernel
# trace of the same command, on the committed library
OUT=gpurun_out/close_r02
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('default', round(d['value']), round(d['ms_per_step'],1), d['roofline']['frac'], d['config'].get('route'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
