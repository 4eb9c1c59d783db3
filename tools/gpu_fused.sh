#!/bin/bash
# The fused layer kernel k_gl4f (SD_OPT_SPLIT_ROUTE 6): its bitwise tests against
# the tiled split route, then same-box bench A/B against the default route (tools/gpu_ab.sh).
# usage: bash tools/gpu_fused.sh <tag> [extra gpu_ab.sh arguments]
TAG=${1:-fused}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread \
    -k "fused_layer or tiled_split or config2_as_benched or f16_range" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "amass16|" "amass16|--option split_route=6" "amass16|--option split_route=6 --option row_chains=1" \
    "amass16|--option split_route=6 --option row_chains=2" "$@"
