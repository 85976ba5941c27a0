# round-5 verify: the driver's default bench command and the VALU-bound
# configs on the committed profiles/pmc_summary.json (the tree's build), so each
# line carries traffic and the one-run VALU fraction as the round-end bench will
mkdir -p gpurun_out/verify
timeout -k 10 300 python bench.py > gpurun_out/verify/bench_default.json 2> gpurun_out/verify/bench_default.err &&
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/verify/bench_c4.json 2> gpurun_out/verify/bench_c4.err &&
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/verify/bench_c5.json 2> gpurun_out/verify/bench_c5.err &&
timeout -k 10 300 python bench.py --op polymul --param p-III-8192 --batch 131072 --no-cpu-baseline > gpurun_out/verify/benchm_8192.json 2> gpurun_out/verify/benchm_8192.err &&
timeout -k 10 300 python bench.py --config 1 --steps 1000 --no-cpu-baseline > gpurun_out/verify/bench_c1.json 2> gpurun_out/verify/bench_c1.err
