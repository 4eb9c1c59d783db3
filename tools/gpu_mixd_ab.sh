# Same-box A/B of the k_gl5_mixd forms (SKELDIFF_V5_MIXD, sd_graph_linear_v5.hip): the config-3 GPU tests under
# each form in MIXD_TEST, then two rounds of bench lines of config 3 per form in MIXD_CFGS (0 = the default).
mkdir -p gpurun_out/mixd
for m in ${MIXD_TEST:-1 2}; do
  SKELDIFF_V5_MIXD=$m timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mano or config3" > gpurun_out/mixd/pytest_$m.txt 2>&1 || { echo "pytest mixd=$m failed"; tail -5 gpurun_out/mixd/pytest_$m.txt; exit 1; }
  tail -1 gpurun_out/mixd/pytest_$m.txt
done
B="--config mano51 --no-cpu-baseline --no-exact-line --profile-reps 1 --steps 3 --warmup 1"
for i in 1 2; do
  for m in ${MIXD_CFGS:-0 1 2}; do
    SKELDIFF_V5_MIXD=$m timeout -k 10 300 python bench.py $B > gpurun_out/mixd/b.json 2>> gpurun_out/mixd/b.err || { echo "bench failed $m"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/mixd/b.json'));print('mixd=$m', round(d['value'],1), 'futures/s')"
  done
done
