set -o pipefail
# large-n launch shapes: products per wave capped at 16 (a_base) vs 32 / 64 (fewer workgroup drains per CU)
O=gpurun_out/r4t; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
NTT_AMD_LIB=$PWD/$L/p64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "not expired" -x -q --timeout 150 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/p32.so $L/p64.so --param p-III-4096 --batch 262144 --ops mul --rounds 9 > $O/ab_m4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/p32.so $L/p64.so --param p-III-8192 --batch 131072 --ops mul --rounds 9 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/p32.so $L/p64.so --param p-III-4096 --batch 524288 --ops fwd,inv --inplace --rounds 9 > $O/ab_l4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/p32.so $L/p64.so --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 > $O/ab_l8192.log 2>&1 || exit 1
echo done
