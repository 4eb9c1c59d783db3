mkdir -p gpurun_out/r06d
timeout -k 10 120 ./tools/gl4t_rt_probe 200 > gpurun_out/r06d/probe.txt 2>&1; echo probe rc=$?
bash tools/gpu_final.sh r06d
