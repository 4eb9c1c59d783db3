set -u
bash tools/gpu_check.sh && PMC=1 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline" bash tools/profile.sh r01_v3
