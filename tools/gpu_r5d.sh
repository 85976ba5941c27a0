# round 5: headline transforms with ascending store addresses (NTT_STORE_SEQ)
# against the product build, one process, interleaved
bash tools/gpu_session.sh abx
