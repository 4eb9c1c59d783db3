for cfg in 0 100; do
  SKELDIFF_GL4_CFG=$cfg timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/attn_$cfg.log 2>&1 || exit $?
  echo "cfg=$cfg"; python -c "
import json; r=json.loads([l for l in open('gpurun_out/attn_$cfg.log') if l.startswith('{')][-1]); print(r['value'], r['kernels_per_denoise_step_ms'])"
done
