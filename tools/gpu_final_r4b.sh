# round-4 measurement, part 2: rocprofv3 kernel stats, FETCH/WRITE PMC, VALU counters
bash tools/gpu_session.sh prof_c2 prof_c3 prof_c4 prof_c5 profl_4096 profl_8192 profm_4096 profm_8192 pmc_c2 pmc_c3 pmc_c4 pmc_c5 pmcl_4096 pmcl_8192 pmcm_4096 pmcm_8192 valu_c4 valu_c5 valum_4096 valum_8192
