#!/bin/bash
# rocprofv3 profile of the bench command (run on the GPU box via gpurun):
#   1. --kernel-trace --stats  on the default workload (T=100)    -> per-kernel average durations
#   2. --pmc FETCH_SIZE        (separate pass, short T)            -> HBM read bytes (x2 on gfx950)
#   3. --pmc WRITE_SIZE        (separate pass, short T)            -> HBM write bytes
# Counters are collected in their own runs, never combined with sys/runtime traces.  The PMC
# passes run T=4 (per-launch traffic does not depend on T) so they finish in seconds.
# Output: gpurun_out/prof_<tag>/...
set -u
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
PMC_ARGS=${BENCH_PMC_ARGS:-"--T 4 --steps 1 --warmup 1 --no-cpu-baseline --no-graph --profile-reps 1"}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace_rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
      python3 bench.py $PMC_ARGS > $OUT/pmc_fetch.log 2>&1
  rc=$?; echo "pmc_fetch_rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
      python3 bench.py $PMC_ARGS > $OUT/pmc_write.log 2>&1
  rc=$?; echo "pmc_write_rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
