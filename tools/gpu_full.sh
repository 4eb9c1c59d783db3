mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --precision half --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_a16_half.log 2>&1 || { tail -20 gpurun_out/bench_a16_half.log; exit 1; }
grep '^{' gpurun_out/bench_a16_half.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("amass16 half", d["value"], d["ms_per_step"], d["kernels_per_denoise_step_ms"])'
