#!/bin/bash
# A round's closing measurements on one box: the default bench line (with the CPU baseline), the
# rocprofv3 profile of it (tools/prof_bench.sh: kernel trace + FETCH / WRITE / SQ passes), the
# config-3 line, and the k_gemm kernel trace + LDS-conflict pass of the training step.
# usage: bash tools/gpu_close.sh <tag>      (outputs under gpurun_out/<tag>, gpurun_out/prof_<tag>)
TAG=${1:-close}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/prof_bench.sh $TAG || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT/ktr $OUT/pmc_kgemm
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktr -o run -- \
    python3 tools/bench_train.py --J 16 --rows 1024 --steps 5 --warmup 2 --modes hip > $OUT/ktr.log 2>&1
rc=$?; echo "train trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv \
    -d $OUT/pmc_kgemm/p1 -o run -- python3 tools/bench_train.py --J 16 --rows 1024 --steps 1 --warmup 1 --modes hip \
    > $OUT/pmc_kgemm/p1.log 2>&1
rc=$?; echo "k_gemm pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config mano51 --no-cpu-baseline --no-exact-line > $OUT/bench_mano51.json 2> $OUT/bench_mano51.err
rc=$?; echo "mano51 rc=$rc"; exit $rc
