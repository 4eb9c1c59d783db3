#!/bin/bash
# Round-3 closing run: smoke, GPU suite, default bench line + rocprofv3 profile (+ the MANO shard's),
# one line per config.
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_session.sh ${1:-r03d} mano51 || exit $?
bash tools/bench_configs.sh configs_${1:-r03d}
