#!/bin/bash
# Small-batch route (v5 for <= 128 rows): full GPU suite, then config 4 and config 2 benches.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config h36m_t1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_h36m_t1000.log 2>&1
rc=$?; echo "cfg4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/cfg_h36m_t1000.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg4', round(r['value'],2))"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('cfg2', round(r['value'],1))"
