set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_parity_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_head.so $L/b_wt.so --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 41 > $O/ab_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_head.so $L/b_wt.so --param p-I --ops fwd,inv,mul --inplace --rounds 7 > $O/ab_p1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_head.so $L/b_wt.so $L/c_w8.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 7 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_head.so $L/b_wt.so --param p-III-4096 --batch 262144 --ops mul,mulntt --rounds 7 > $O/ab_m4096.log 2>&1 || exit 1
bash tools/gpu_session.sh pmc_c2 bench_c2 || exit 1
cp gpurun_out/pmc_summary.json gpurun_out/session.log gpurun_out/bench_c2.log $O/
echo done
