# round 5: bench lines of configs 1 and 2 with the latency kernels
bash tools/gpu_session.sh bench_c1 bench_c2
