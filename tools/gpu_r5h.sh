# round 5: small-batch latency of the transforms (tools/latency.py), and the
# kernel durations of the same run under rocprofv3
mkdir -p gpurun_out
timeout -k 10 200 python tools/latency.py > gpurun_out/latency.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_latency -o run -- python3 tools/latency.py --rounds 1 --steps 50 > gpurun_out/latency_prof.log 2>&1
