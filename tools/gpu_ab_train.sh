#!/bin/bash
# Same-box A/B of a training-kernel switch read at library load (default: SKELDIFF_GEMM_RING 0 vs 1),
# hip mode of tools/bench_train.py, alternating A B A B.  usage: bash tools/gpu_ab_train.sh [VAR] [J]
VAR=${1:-SKELDIFF_GEMM_RING}
J=${2:-16}
OUT=gpurun_out/ab_train
mkdir -p $OUT
for rep in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python3 tools/bench_train.py --J $J --modes hip --steps 20 > $OUT/${VAR}_${v}_$rep.json 2> $OUT/${VAR}_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$VAR=$v rc=$rc"; exit $rc; }
    echo "$VAR=$v rep $rep: $(python3 -c "import json; print(round(json.load(open('$OUT/${VAR}_${v}_$rep.json'))['hip']['ms_per_step'], 3))") ms"
  done
done
