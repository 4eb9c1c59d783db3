#!/bin/bash
# Round evidence: smoke + GPU tests + default bench (with CPU baseline), then the rocprof
# kernel-trace summary and PMC traffic passes for profiles/<tag>.
set -u
TAG=${1:-r01}
bash tools/gpu_check.sh && PMC=1 bash tools/profile.sh $TAG
