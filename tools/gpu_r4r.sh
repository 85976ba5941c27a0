set -o pipefail
# poly_mul with compact twiddle tables on 8-wave workgroups, 2 per CU (r_cmp) vs the final build (a_base)
O=gpurun_out/r4r; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
NTT_AMD_LIB=$PWD/$L/r_cmp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/a_base.so $L/r_cmp.so --ops mul,mulntt --rounds 9 > $O/ab_p3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/a_base.so $L/r_cmp.so --param p-I --ops mul,mulntt --rounds 9 > $O/ab_p1.log 2>&1 || exit 1
echo done
