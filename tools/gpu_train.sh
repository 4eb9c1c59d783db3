#!/bin/bash
# training-side check: GPU training tests, the training-step bench (J = 16 / 21) and a kernel trace
set -o pipefail
OUT=gpurun_out/${1:-train}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_training.py tests/test_best_of_k.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for J in 16 21; do
  timeout -k 10 300 python -u tools/bench_train.py --J $J --rows 1024 --steps 10 --warmup 3 > $OUT/train$J.json 2> $OUT/train$J.err
  rc=$?; echo "train J=$J rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/train$J.json'));print(round(d['hip']['ms_per_step'],2), round(d['torch_ops_same_gpu']['ms_per_step'],2), round(d['speedup'],2))")"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 tools/bench_train.py --J 16 --rows 1024 --steps 3 --warmup 1 --modes hip > $OUT/prof.log 2>&1
echo "prof rc=$?"
