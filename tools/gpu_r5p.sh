# round 5: small-batch latency of the n = 4096 / 8192 sets (batch kernels only)
mkdir -p gpurun_out
timeout -k 10 200 python tools/latency.py --params p-III-4096,p-III-8192 --batches 1,16,256 --rounds 3 > gpurun_out/lat_large.log 2>&1
