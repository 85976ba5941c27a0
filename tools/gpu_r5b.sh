# round 5: Nussbaumer with the next unit's loads software-pipelined
# (ppw 1 / 4 / 16) and the n = 4096 / 8192 inverse with the next polynomial's
# loads in its last stage (8 / 12 waves at n = 8192), against the r04
# kernels (a_base), one process, interleaved
bash tools/gpu_session.sh abnus nusstamps
