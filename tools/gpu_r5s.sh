# round 5: the Python wrapper's cheaper per-call checks: every GPU test, then
# config 1's bench line (one polynomial per call)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 &&
bash tools/gpu_session.sh bench_c1
