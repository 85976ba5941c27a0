set -o pipefail
# one copy of the work loop's body (no peeled first unit): half the code of every kernel
O=gpurun_out/r4h; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib
A="$L/libqtesla_ntt.so $L/ab/h_nopeel.so"
timeout -k 10 200 python -u tools/ab.py $A --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 > $O/ab_l8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $A --param p-III-4096 --batch 262144 --ops mul,mulntt --rounds 9 > $O/ab_m4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $A --param p-III-4096 --batch 524288 --ops fwd,inv --inplace --rounds 9 > $O/ab_l4096.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $A --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 9 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $A --ops fwd,inv,mul,mulntt --inplace --rounds 9 > $O/ab_p3.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $A --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 41 > $O/ab_c2.log 2>&1 || exit 1
echo done
