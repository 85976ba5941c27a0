# round 5: latency kernels at every batch (NTT_LAT_MAX huge) against the
# batch kernels (NTT_LAT_MAX=0): the crossover for NTT_LAT_MAX
mkdir -p gpurun_out
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/a_nolat.so --batches 128,256,512,1024,2048 --rounds 3 > gpurun_out/latx_a_nolat.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/c_latbig.so --batches 128,256,512,1024,2048 --rounds 3 > gpurun_out/latx_c_latbig.log 2>&1
