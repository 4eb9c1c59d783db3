run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cp_$name.log 2>&1 || { tail -20 gpurun_out/cp_$name.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/cp_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_per_denoise_step_ms"]["graph_linear"])')"
}
run c3_811 SKELDIFF_GL4_CFG=811
run c1_811 SKELDIFF_GL4_CFG=811 SKELDIFF_CHAINS=1
