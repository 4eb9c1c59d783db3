#!/bin/bash
# Route / row-chain sweep only (tools/sweep_routes.py); env SWEEP_ROUTES / SWEEP_CHAINS narrow it.
# usage: bash tools/gpu_sweep.sh <tag> [config[:batch][:T] ...]
TAG=${1:-sweep}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u tools/sweep_routes.py "$@" > gpurun_out/$TAG/sweep.log 2>&1
rc=$?
echo "sweep rc=$rc"
python3 - gpurun_out/$TAG/sweep.log <<'PY'
import json, sys
from collections import defaultdict
t = defaultdict(dict)
for l in open(sys.argv[1]):
    if l.startswith("{"):
        r = json.loads(l)
        t[r["config"]][(r["split_route"], r["row_chains"])] = r["futures_per_s"]
for c, v in t.items():
    print(c, " ".join(f"r{k[0]}c{k[1]}={x:.0f}" for k, x in sorted(v.items())))
PY
exit $rc
