set -o pipefail
# n = 8192 poly_mul in the incomplete domain (compact per-sub-tree tables, 16 waves) vs b_head;
# config-2 launch shape: >= 4 (ppw 4) / 8 (ppw 2) / 16 (ppw 1) workgroups per CU
O=gpurun_out/r4k; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
NTT_AMD_LIB=$PWD/$L/ab/k_inc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/b_head.so $L/ab/k_inc.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 9 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/ab/k_inc.so $L/ab/l_wg8.so $L/ab/m_wg16.so --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 41 > $O/ab_c2.log 2>&1 || exit 1
echo done
