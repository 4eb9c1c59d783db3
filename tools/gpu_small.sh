mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -30 gpurun_out/small_tests.log; exit 1; }
tail -1 gpurun_out/small_tests.log
for cfg in h36m_t1000 amass16; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sm_$cfg.log 2>&1 || { tail -20 gpurun_out/sm_$cfg.log; exit 1; }
  echo "$cfg $(grep '^{' gpurun_out/sm_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
