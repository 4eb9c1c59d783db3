#!/bin/bash
# Row-chain experiment: chain-invariance tests, then bench at SKELDIFF_CHAINS = 1 2 3 4
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "row_chains or full_size or graph_replay or row0" > gpurun_out/chains_tests.log 2>&1 || { tail -30 gpurun_out/chains_tests.log; exit 1; }
tail -3 gpurun_out/chains_tests.log
for n in ${CHAINS:-1 2 3 4}; do
  SKELDIFF_CHAINS=$n timeout -k 10 240 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/chains_$n.log 2>&1 || { tail -20 gpurun_out/chains_$n.log; exit 1; }
  echo "chains=$n $(grep '^{' gpurun_out/chains_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
