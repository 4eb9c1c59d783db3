#!/bin/bash
# SQ / TCC counters for one graph-linear shape (tools/bench_gl.py SHAPE=...), one counter group
# per rocprofv3 pass (--pmc only, never combined with sys/runtime traces).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_gl_${TAG:-x}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/bench_gl.py > $OUT/p$i.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
  echo "pass $i ($grp) rc=$rc"
done
exit 0
