set -o pipefail
# wave-per-polynomial n = 4096 products (ntt_big.hpp) vs the multi-wave ones (b_head);
# n = 8192 product with the phase pin (115 VGPRs) vs b_head (168 + 6 spilled)
O=gpurun_out/r4f; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so $L/ab/e_bm8.so --param p-III-4096 --batch 262144 --ops mul,mulntt --rounds 9 > $O/ab_m4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 9 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so --param p-III-4096 --batch 524288 --ops fwd,inv --inplace --rounds 9 > $O/ab_l4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 > $O/ab_l8192.log 2>&1 || exit 1
echo done
