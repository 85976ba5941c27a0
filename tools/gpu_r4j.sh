set -o pipefail
# Nussbaumer at 2.5 waves/SIMD (X / Y transposes in turn, half of X-hat stashed in LDS, 32-bit reductions, per-phase lane geometry)
O=gpurun_out/r4j; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_nussbaumer.py -x -q --timeout 150 --timeout-method thread > $O/pytest_nus.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/ab/b_head.so $L/ab/j_nus3.so --ops nus,nusm32 --rounds 7 > $O/ab_nus_p3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/ab/b_head.so $L/ab/j_nus3.so --param p-I --ops nus,nusm32 --rounds 7 > $O/ab_nus_p1.log 2>&1 || exit 1
echo done
