#!/bin/bash
# One bench line per BASELINE config shape (1 GPU), for DESIGN.md / profiles.
mkdir -p gpurun_out
for cfg in ${CFGS:-amass16 amass21 freeman17 freeman17_half mano51 h36m_t1000}; do
  steps=2; [ $cfg = h36m_t1000 ] && steps=3
  timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$cfg.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/cfg_$cfg.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['config']['workload'], '|', round(r['value'],1), r['unit'], '| ms/sample', round(r['ms_per_step'],2), '| GL TF/s', round(r['roofline']['achieved'],1), '|', r['arithmetic'][:40])"
done
