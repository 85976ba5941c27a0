# round-4 measurement, part 1: GPU tests, smoke, bench lines (with CPU baselines); then the no-peel A/B
bash tools/gpu_session.sh pytest smoke bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 benchl_4096 benchl_8192 benchm_4096 benchm_8192 && bash tools/gpu_r4h.sh
