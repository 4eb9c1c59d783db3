# half precision mode: quality gate tests + config-5 bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_precision.py tests/test_checkpoint.py -x -q --timeout 120 --timeout-method thread > gpurun_out/half_tests.log 2>&1 || { tail -40 gpurun_out/half_tests.log; exit 1; }
tail -1 gpurun_out/half_tests.log
timeout -k 10 300 python -u bench.py --config freeman17_half --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_half.log 2>&1 || { tail -20 gpurun_out/bench_half.log; exit 1; }
grep '^{' gpurun_out/bench_half.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("freeman17_half", d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])'
timeout -k 10 300 python -u bench.py --config freeman17 --T 10 --batch 1377 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_f17.log 2>&1 || { tail -20 gpurun_out/bench_f17.log; exit 1; }
grep '^{' gpurun_out/bench_f17.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("freeman17 f32 same shape", d["value"], d["ms_per_step"])'
