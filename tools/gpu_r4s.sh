set -o pipefail
# n = 8192 poly_mul (incomplete domain) on two 8-wave workgroups per CU (s_inc8) vs one 16-wave (a_base)
O=gpurun_out/r4s; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
NTT_AMD_LIB=$PWD/$L/s_inc8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/s_inc8.so --param p-III-8192 --batch 131072 --ops mul --rounds 11 > $O/ab_m8192.log 2>&1 || exit 1
echo done
