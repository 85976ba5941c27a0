# round 5: latency kernels at n = 4096 / 8192 (ntt_lat.hpp R = 2 groups per
# thread at n = 8192): the large-set and parity GPU tests, then the crossover
# against the batch kernels
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_large.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/a_nolat.so --params p-III-8192 --batches 1,64,256,512 --rounds 3 > gpurun_out/latm_a_nolat.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/c_latbig.so --params p-III-8192 --batches 1,64,256,512 --rounds 3 > gpurun_out/latm_c_latbig.log 2>&1
