# round-5 first GPU session: the cleaned-up build (asm-identical to r04's
# kernels) through the GPU tests (incl. the new config-4/5 two-rank bench
# tests) and smoke; the headline line with its new pattern floor; the VALU
# cost table with every emitted opcode; Nussbaumer's and the n = 8192
# transforms' SQ stall counters; the n = 8192 occupancy / stagger A/B
bash tools/gpu_session.sh pytest smoke bench_c3 valucost sq_c5 sqb_c5 sql_8192 abl_8192 listpmc
