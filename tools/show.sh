#!/bin/bash
tail -1 gpurun_out/pytest_q.log; grep -v amdgpu gpurun_out/bench_gl.log
python - <<'PY'
import json
r = json.loads(open('gpurun_out/bench_q.log').read().strip().splitlines()[-1])
print(round(r['value'], 1), 'fut/s', round(r['ms_per_step'], 1), 'ms/sample', {k: round(v, 3) for k, v in r['kernels_per_denoise_step_ms'].items()}, round(r['roofline']['achieved'], 2), 'TF')
PY
