#!/bin/bash
# rocprofv3 trace + PMC traffic passes of the default bench command on the closing code (tiled
# route for config 2), summarised into profiles/r02t_summary.md + profiles/pmc_traffic.json
bash tools/profile.sh r02t || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r02t r02t > /dev/null && echo summary ok
