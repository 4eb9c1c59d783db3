mkdir -p gpurun_out
for n in 1 2 4; do
  SKELDIFF_CHAINS=$n timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-graph > gpurun_out/eager_$n.log 2>&1 || { tail -20 gpurun_out/eager_$n.log; exit 1; }
  echo "eager chains=$n $(grep '^{' gpurun_out/eager_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
