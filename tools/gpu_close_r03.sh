#!/bin/bash
# Round-3 closing run: GPU suite, default bench line + rocprofv3 profile, one line per config.
bash tools/gpu_session.sh ${1:-r03c} || exit $?
bash tools/bench_configs.sh configs_${1:-r03c}
