# round 5: static priority (s_setprio 1) for the second half of the
# workgroup's waves, in poly_mul (MUL_PRIO_HALF) / the transforms
# (NTT_PRIO_HALF), against the tree's build; then configs 1 and 2's bench lines
bash tools/gpu_session.sh abx bench_c1 bench_c2
