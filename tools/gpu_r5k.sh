# round 5: the latency kernels in the product build: every GPU test, the
# Python-path latency (tools/latency.py) and the native C-ABI per-call latency
# (ntt_main -speedgpu 12) at batch 1 and 64
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --batches 1,64,1024 --rounds 3 > gpurun_out/lat_product.log 2>&1 &&
for p in p-I p-III; do for b in 1 64; do
  timeout -k 10 60 ./ntt-gpu-qtesla_amd/bin/ntt_main -speedgpu 12 -param $p -batch $b > gpurun_out/native_lat_${p}_$b.log 2>&1 || exit 1
done; done
