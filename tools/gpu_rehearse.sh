# multi-rank bench rehearsal on ONE GPU (gloo): barrier, broadcast_state, MAX all-reduce, rank-0 JSON
mkdir -p gpurun_out
SKELDIFF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/rehearse.log 2>&1 || { tail -30 gpurun_out/rehearse.log; exit 1; }
grep '^{' gpurun_out/rehearse.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("n_gpus", d["n_gpus"], "value", d["value"], "ms", d["ms_per_step"], d["config"]["parallelism"])'
