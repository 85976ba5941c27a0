# round 5: rocprofv3 kernel statistics of the latency kernels (batch 1 and 64,
# every parameter set; graph replay off so the trace sees plain launches)
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lat -o run -- python3 tools/latency.py --params ref,p-I,p-III,p-III-4096,p-III-8192 --batches 1,64 --rounds 1 --steps 200 --no-graph > gpurun_out/prof_lat.log 2>&1
