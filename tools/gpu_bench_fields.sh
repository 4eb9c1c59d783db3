#!/bin/bash
# bench.py JSON sanity per route: value, route, row chains, roofline kernel and fraction
for c in amass16 freeman17 mano51 h36m_t1000; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-exact-line > gpurun_out/bj_$c.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/bj_$c.json'));print('$c', round(d['value'],1), d['config']['route'], d['config']['row_chains'], d['roofline']['kernel'][:40], round(d['roofline']['frac'],3))"
done
