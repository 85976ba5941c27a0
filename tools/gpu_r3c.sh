set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so
for spec in "polymul p-III-4096 262144" "polymul_ntt p-III-4096 262144" "polymul p-III-8192 131072" "polymul_ntt p-III-8192 131072"; do
  set -- $spec
  timeout -k 10 240 python -u bench.py --op $1 --param $2 --batch $3 --steps 20 --warmup 3 --cpu-seconds 8 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || exit 1
  tail -c 600 $O/bench_$1_$2.json; echo
done
timeout -k 10 120 python -u tools/ab.py $L --param p-III-4096 --batch 262144 --ops bitrev,fwdbr,invbr,fwd,inv --inplace --rounds 5 > $O/ab_bitrev_4096.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ab.py $L --param p-III-8192 --batch 131072 --ops bitrev,fwdbr,invbr,fwd,inv --inplace --rounds 5 > $O/ab_bitrev_8192.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_mul4096 -o run -- python3 bench.py --op polymul --param p-III-4096 --batch 262144 --steps 10 --warmup 2 --no-cpu-baseline --no-check > $O/prof_mul4096.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_mul8192 -o run -- python3 bench.py --op polymul --param p-III-8192 --batch 131072 --steps 10 --warmup 2 --no-cpu-baseline --no-check > $O/prof_mul8192.log 2>&1 || exit 1

echo done
