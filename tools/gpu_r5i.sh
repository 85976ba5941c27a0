# round 5: small-batch latency kernels (csrc/ntt_lat.hpp): parity tests, then
# tools/latency.py on the build without them (NTT_LAT_MAX=0) and with them
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/a_nolat.so --batches 1,64,256,1024,4096 --rounds 3 > gpurun_out/lat_a_nolat.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/b_lat.so --batches 1,64,256,1024,4096 --rounds 3 > gpurun_out/lat_b_lat.log 2>&1
