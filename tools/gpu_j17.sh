mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/j17_$name.log 2>&1 || { tail -20 gpurun_out/j17_$name.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/j17_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_precision.py -x -q --timeout 120 --timeout-method thread -k "freeman17 or ragged or row_chains" > gpurun_out/j17_tests.log 2>&1 || { tail -40 gpurun_out/j17_tests.log; exit 1; }
tail -1 gpurun_out/j17_tests.log
run half812 --config freeman17_half
SKELDIFF_GL4_CFG=821 run half821 --config freeman17_half
run f32_812 --config freeman17
SKELDIFF_GL4_CFG=821 run f32_821 --config freeman17
