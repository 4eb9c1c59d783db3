#!/bin/bash
# Round-2 (second session) measurement: full GPU suite on the committed library, the default bench
# line, and the configs today's kernels touch (MANO J = 51 / 52, config 4 on the split route)
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('default', round(d['value']), round(d['ms_per_step'],1), d['roofline']['frac'])"
CFGS="mano51 mano52 h36m_t1000" bash tools/bench_configs.sh || exit 1
cp gpurun_out/cfg_*.log $OUT/
