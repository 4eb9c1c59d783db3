mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "2812 or three_stage" > gpurun_out/xp2_tests.log 2>&1 || { tail -30 gpurun_out/xp2_tests.log; exit 1; }
tail -1 gpurun_out/xp2_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cp_$name.log 2>&1 || { tail -20 gpurun_out/cp_$name.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/cp_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_per_denoise_step_ms"]["graph_linear"])')"
}
run c3_2812 SKELDIFF_GL4_CFG=2812
run c1_2812 SKELDIFF_GL4_CFG=2812 SKELDIFF_CHAINS=1
run c1_812 SKELDIFF_GL4_CFG=812 SKELDIFF_CHAINS=1
