#!/bin/bash
# Round-2 closing session: full GPU suite on the committed library, the default bench line, one
# line per BASELINE config, rocprofv3 kernel stats of the FreeMan J = 17 tiled route
OUT=gpurun_out/final_r02
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('default', round(d['value']), round(d['ms_per_step'],1), round(d['roofline']['frac'],3))"
CFGS="amass21 freeman17 freeman17_half freeman17_bf16 mano51 mano52 h36m_t1000" bash tools/bench_configs.sh || exit 1
cp gpurun_out/cfg_*.log $OUT/
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_freeman17 -o run -- python3 bench.py --config freeman17 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
