mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_precision.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j_tests.log 2>&1 || { tail -30 gpurun_out/j_tests.log; exit 1; }
tail -1 gpurun_out/j_tests.log
for cfg in amass21 freeman17 amass16; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/j_$cfg.log 2>&1 || { tail -20 gpurun_out/j_$cfg.log; exit 1; }
  echo "$cfg $(grep '^{' gpurun_out/j_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 400 python -u tools/eval_pipeline.py 256 10 > gpurun_out/evalp2.log 2>&1 && tail -1 gpurun_out/evalp2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("e2e", d["value"], d["stage_ms"])'
