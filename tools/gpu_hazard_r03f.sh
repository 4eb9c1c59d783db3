#!/bin/bash
# DESIGN.md §4c, round 3 (sixth run): the CU-sharing build with packed-FP32 codegen disabled
# (libskeldiff_nopk.so) vs the same build with it (libskeldiff_share.so), three tiled row chains
# sharing CUs, tools/tiled_check.py at T = 4 (x3 each), then config-2 bench lines of both on
# the tiled route with three chains (and the product library as shipped)
OUT=gpurun_out/hazard_r03
mkdir -p $OUT
export TILED_RUNS="one-kernel,tiled 3 chains"
for lib in nopk share nopk nopk; do
    SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_$lib.so timeout -k 10 200 python -u tools/tiled_check.py amass16 4 64 > $OUT/pk_$lib.log 2>&1
    rc=$?
    echo "$lib rc=$rc: $(grep 'tiled 3 chains' $OUT/pk_$lib.log | sed 's/first rows.*//' | tr '\n' ' ')"
    [ $rc -le 1 ] || exit 1
done
for lib in nopk share; do
    SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_$lib.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 \
        --no-cpu-baseline --no-exact-line --option split_route=3 --option row_chains=3 > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err
    echo "bench $lib rc=$?: $(python -c "import json;d=json.load(open('$OUT/bench_$lib.json'));print(round(d['value']),d['ms_per_step'])")"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-line > $OUT/bench_prod.json 2> $OUT/bench_prod.err
echo "bench product rc=$?: $(python -c "import json;d=json.load(open('$OUT/bench_prod.json'));print(round(d['value']),d['ms_per_step'])")"
