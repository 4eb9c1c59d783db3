set -e
GRAPHS="0 1" NCH="2 3" timeout -k 10 300 python -u tools/chain_debug.py 100
GRAPHS="1" NCH="3" timeout -k 10 300 python -u tools/chain_debug.py 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -5 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
bash tools/gpu_chain_perf.sh
