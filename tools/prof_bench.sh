#!/bin/bash
# rocprofv3 profile of the bench command (on the GPU box via gpurun), one pass per counter group:
#   trace  --kernel-trace --stats, the bench as run by the driver (per-kernel average durations)
#   fetch  --pmc FETCH_SIZE   (HBM read bytes; x2 on gfx950, MI355X_MICROARCH.md §HBM)
#   write  --pmc WRITE_SIZE
#   sq     --pmc SQ_* MFMA-busy / stall counters + GRBM_GUI_ACTIVE
# PMC passes run T = 4 on one row chain (per-launch traffic depends on neither).  Summary:
# tools/prof_bench.py.
# usage: bash tools/prof_bench.sh <tag> [extra bench args]
set -u
TAG=${1:-r03}
shift
EXTRA="$*"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-line $EXTRA > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; rm -f $OUT/trace/run_kernel_trace.csv  # stats kept; gpurun_out is capped at 64 MiB
[ $rc -eq 0 ] || exit $rc
# one row chain: every dispatch covers the full batch, as the roofline's per-launch timing does
PMC_ARGS="--T 4 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-line --profile-reps 1 --option row_chains=1 $EXTRA"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py $PMC_ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
