set -o pipefail
# n = 4096 poly_mul on compact tables and two 4-wave workgroups per CU (c4) vs one 8-wave workgroup (a_base)
O=gpurun_out/r4u; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
NTT_AMD_LIB=$PWD/$L/c4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "not expired" -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/c4.so --param p-III-4096 --batch 262144 --ops mul --rounds 11 > $O/ab_m4096.log 2>&1 || exit 1
echo done
