set -o pipefail
# scheduler flag A/B: -mllvm -amdgpu-use-amdgpu-trackers (q_trk) vs the final build (a_base)
O=gpurun_out/r4q; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
timeout -k 10 300 python -u tools/ab.py $L/a_base.so $L/q_trk.so --ops fwd,inv,mul,mulntt,nus --inplace --rounds 7 > $O/ab_p3.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/q_trk.so --param p-I --batch 65536 --ops fwd --inplace --rounds 41 > $O/ab_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_base.so $L/q_trk.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 7 > $O/ab_m8192.log 2>&1 || exit 1
echo done
