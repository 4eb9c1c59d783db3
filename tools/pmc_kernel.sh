#!/bin/bash
# SQ / TCC / GRBM counters of any command, one counter group per rocprofv3 pass (--pmc only,
# never combined with sys / runtime traces; at most 8 SQ / 4 TCC / 2 GRBM counters per pass).
# usage: TAG=<tag> [PMC_GROUPS="CTR CTR ...;CTR ..."] bash tools/pmc_kernel.sh python3 <script> [args]
#   PMC_GROUPS: ';'-separated counter groups, one pass each (default: the stall / LDS / traffic set)
# summary: python tools/pmc_report.py --kernel <regex> --dir gpurun_out/pmc_<tag> <tag>
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p $OUT
i=0
if [ -n "${PMC_GROUPS:-}" ]; then IFS=';' read -r -a GRPS <<< "$PMC_GROUPS"; else GRPS=(
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA" \
           "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"); fi
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -le 1 ] || exit $rc
done
exit 0
