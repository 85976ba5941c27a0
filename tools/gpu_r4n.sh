set -o pipefail
# n = 8192 poly_mul_ntt at 16 waves with the bit-5 pairs from __constant__ (n_bit5u) vs 12 waves (k_inc)
O=gpurun_out/r4n; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
NTT_AMD_LIB=$PWD/$L/ab/n_bit5u.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/k_inc.so $L/ab/n_bit5u.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 9 > $O/ab_m8192.log 2>&1 || exit 1
echo done
