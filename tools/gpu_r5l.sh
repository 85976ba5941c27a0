# round 5: small-batch products (k_poly_mul_lat): every GPU test, then the
# crossover of the latency kernels (transforms and products) against the
# batch kernels, and the native per-call latency
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/a_nolat.so --batches 1,64,256,512,1024,2048 --rounds 3 > gpurun_out/laty_a_nolat.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/ab/c_latbig.so --batches 1,64,256,512,1024,2048 --rounds 3 > gpurun_out/laty_c_latbig.log 2>&1 &&
for p in p-I p-III; do for b in 1 64; do
  timeout -k 10 60 ./ntt-gpu-qtesla_amd/bin/ntt_main -speedgpu 12 -param $p -batch $b > gpurun_out/native_lat_${p}_$b.log 2>&1 || exit 1
done; done
