# round 5: last check of the tree as committed: smoke, the driver's default
# bench command, config 4
bash tools/gpu_session.sh smoke bench bench_c4
