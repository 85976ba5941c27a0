# round 5: the latency switch's boundary test, the wrapper's own per-call
# cost (tools/latency.py poly_ntt vs poly_ntt_ctypes), then the verify bench
# lines on the committed summary (tools/gpu_verify_r5.sh)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "latency_switch or host_driver" --timeout 120 --timeout-method thread > gpurun_out/boundary.log 2>&1 &&
timeout -k 10 200 python tools/latency.py --batches 1 --rounds 5 > gpurun_out/lat_ctypes.log 2>&1 &&
bash tools/gpu_verify_r5.sh
