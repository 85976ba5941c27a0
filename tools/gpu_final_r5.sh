# round-5 measurement of the tree's build, one call: GPU tests, smoke, bench
# lines (CPU baselines; config 3 with its pattern floor), rocprofv3 kernel
# stats, FETCH/WRITE PMC and VALU counters of every workload, config 5's SQ
# stall counters (tools/archive_final.sh + valu_summary.py turn them into
# profiles/r05/final/ and profiles/pmc_summary.json)
bash tools/gpu_session.sh pytest smoke bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 benchl_4096 benchl_8192 benchm_4096 benchm_8192 \
    prof_c2 prof_c3 prof_c4 prof_c5 profl_4096 profl_8192 profm_4096 profm_8192 \
    pmc_c2 pmc_c3 pmc_c4 pmc_c5 pmcl_4096 pmcl_8192 pmcm_4096 pmcm_8192 valu_c4 valu_c5 valum_4096 valum_8192 sq_c5 sqb_c5
