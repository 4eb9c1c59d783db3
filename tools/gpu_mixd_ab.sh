mkdir -p gpurun_out/mixd
for m in 1 2; do
  SKELDIFF_V5_MIXD=$m timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mano or config3" > gpurun_out/mixd/pytest_$m.txt 2>&1 || { echo "pytest mixd=$m failed"; tail -5 gpurun_out/mixd/pytest_$m.txt; exit 1; }
  tail -1 gpurun_out/mixd/pytest_$m.txt
done
B="--config mano51 --no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
for i in 1 2; do
  for m in 0 1 2; do
    SKELDIFF_V5_MIXD=$m timeout -k 10 300 python bench.py $B > gpurun_out/mixd/b.json 2>> gpurun_out/mixd/b.err || { echo "bench failed $m"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/mixd/b.json'));print('mixd=$m', round(d['value'],1), 'futures/s')"
  done
done
