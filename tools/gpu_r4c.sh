set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
L=ntt-gpu-qtesla_amd/lib/ab
timeout -k 10 200 python -u tools/ab.py $L/a_old.so $L/b_big8.so $L/c_big12.so --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 7 > $O/ab_8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_old.so $L/b_big8.so --param p-III-4096 --batch 524288 --ops fwd,inv --inplace --rounds 7 > $O/ab_4096.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --op fwdinv --param p-III-8192 --batch 262144 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_l8192.json 2>$O/bench_l8192.err || exit 1
timeout -k 10 200 python -u bench.py --op fwdinv --param p-III-4096 --batch 524288 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_l4096.json 2>$O/bench_l4096.err || exit 1
echo done
