set -o pipefail
# round 4 session 2: HEAD (b_head) vs the round-3 final build (a_r3), then the full GPU suite and bench lines
O=gpurun_out/r4e; mkdir -p $O
L=ntt-gpu-qtesla_amd/lib/ab
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_r3.so $L/b_head.so --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 41 > $O/ab_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_r3.so $L/b_head.so --ops fwd,inv,mul,mulntt --inplace --rounds 7 > $O/ab_p3.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_r3.so $L/b_head.so --param p-I --ops fwd,inv,mul,mulntt --inplace --rounds 7 > $O/ab_p1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_r3.so $L/b_head.so $L/c_w8.so --param p-III-8192 --batch 131072 --ops mul,mulntt --rounds 7 > $O/ab_m8192.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab.py $L/a_r3.so $L/b_head.so --param p-III-4096 --batch 262144 --ops mul,mulntt --rounds 7 > $O/ab_m4096.log 2>&1 || exit 1
for c in 2 3 4 5; do k=20; [ $c = 2 ] && k=1000
  timeout -k 10 300 python -u bench.py --config $c --steps $k --warmup 3 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --no-check > $O/prof_c3.log 2>&1 || exit 1
echo done
