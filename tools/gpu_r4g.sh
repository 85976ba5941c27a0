set -o pipefail
# n = 4096 product variants (8 waves / b prefetched / 4 waves); Nussbaumer with
# opaque rotation masks (no v_cndmask) vs b_head; v_cndmask issue cost
O=gpurun_out/r4g; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_nussbaumer.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/libqtesla_ntt.so $L/ab/f_bm8pf.so $L/ab/g_bm4.so --param p-III-4096 --batch 262144 --ops mul,mulntt --rounds 9 > $O/ab_m4096.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so --ops nus,nusm32 --rounds 5 > $O/ab_nus_p3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L/ab/b_head.so $L/libqtesla_ntt.so --param p-I --ops nus,nusm32 --rounds 5 > $O/ab_nus_p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d $O/valucost -o run -- ./ntt-gpu-qtesla_amd/bin/valu_cost 16384 > $O/valucost.log 2>&1 || exit 1
echo done
