#!/bin/bash
# One GPU-box session: each step has its own time limit; a fault / abort /
# timeout ends the session (no further GPU work in this call).
set -u
mkdir -p gpurun_out
run() {
    local name=$1 secs=$2; shift 2
    echo "[$(date +%T)] start $name" | tee -a gpurun_out/session.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session.log
    case $rc in 124|137|134|139|135|136) echo "fatal rc=$rc in $name, stopping"; exit $rc;; esac
    return 0
}
# named step groups: `final` (one round's full measurement of the tree's
# build: GPU tests, smoke, every bench line with its CPU baselines, rocprofv3
# kernel stats, FETCH / WRITE PMC and VALU counters of every workload, config
# 5's SQ counters; tools/archive_final.sh + tools/valu_summary.py turn its
# gpurun_out/ into profiles/<round>/final/ and profiles/pmc_summary.json) and
# `verify` (the default bench and the VALU-bound lines on the committed summary)
steps=()
for step in "$@"; do
    case $step in
        final) steps+=(pytest smoke bench_c1 bench_c2 bench_c3 bench_c4 bench_c5 benchl_4096 benchl_8192 benchm_4096 benchm_8192
                       prof_c2 prof_c3 prof_c4 prof_c5 profl_4096 profl_8192 profm_4096 profm_8192
                       pmc_c2 pmc_c3 pmc_c4 pmc_c5 pmcl_4096 pmcl_8192 pmcm_4096 pmcm_8192 pmcmn_4096 pmcmn_8192
                       valu_c4 valu_c5 valum_4096 valum_8192 valumn_4096 valumn_8192 sq_c5 sqb_c5) ;;
        verify) steps+=(bench_c2 bench_c3 bench_c4 bench_c5 benchl_4096 benchl_8192 benchm_4096 benchm_8192) ;;
        *) steps+=("$step") ;;
    esac
done
for step in "${steps[@]}"; do
    case $step in
        valu)   run valu 60 ./ntt-gpu-qtesla_amd/bin/valu_rates ;;
        smoke)  run smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
        pytest) run pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ;;
        pytestq) run pytest 600 python -m pytest tests -x -q -m "gpu and not slow" ;;
        bench)  run bench 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 8 ;;
        benchq) run bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
        benchmul) run benchmul 300 python bench.py --op polymul --steps 10 --warmup 2 --no-cpu-baseline ;;
        bench1k) run bench1k 300 python bench.py --op fwd --param p-I --batch 65536 --steps 20 --warmup 2 --no-cpu-baseline ;;
        prof)   run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        variants) run variants 300 python tools/variants.py --rounds 5 ;;
        variants1k) run variants1k 300 python tools/variants.py --param p-I --batch 1048576 --rounds 5 ;;
        pmc) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/variants.py --only fwd_full,inv_full,torch_copy --rounds 2 &&
             run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/variants.py --only fwd_full,inv_full,torch_copy --rounds 2 &&
             run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/variants.py --only fwd_full,inv_full --rounds 2 ;;
        ab) for f in ntt-gpu-qtesla_amd/lib/ab/*.so; do b=$(basename $f .so); NTT_AMD_LIB=$PWD/$f run ab_$b 200 python tools/variants.py --rounds 5 --only fwd_full,inv_full,fwd_alu,inv_alu,fwd_mem,inv_mem || exit 1; done ;;
        abx) run abx_p3 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --ops fwd,inv,mul,mulntt --inplace --rounds 7 &&
             run abx_p1 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-I --ops fwd,inv,mul --inplace --rounds 7 &&
             run abx_p1s 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 21 ;;
        absmall) run abs_p1s 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 31 &&
             run abs_p3 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --ops fwd,inv --inplace --rounds 7 ;;
        abmul2) run abm_p3 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --ops mul,mulntt --rounds 7 &&
                run abm_p1 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-I --ops mul,mulntt --rounds 7 ;;
        abnus) run abn_p3 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --ops nus,nusm32 --rounds 5 &&
               run abn_p1 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-I --ops nus,nusm32 --rounds 5 ;;
        abnusref) run abn_ref 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param ref --ops nus --rounds 7 ;;
        cycles) run cycles 120 ./ntt-gpu-qtesla_amd/bin/valu_cycles ;;
        clock) run pmc_clock 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_clock -o run -- python3 tools/variants.py --rounds 2 ;;
        bocc) run bocc 120 ./ntt-gpu-qtesla_amd/bin/bfly_occupancy ;;
        copybw) run copybw 200 ./ntt-gpu-qtesla_amd/bin/copy_bw ;;
        pmcbench) run pmcb_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcb_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check &&
                  run pmcb_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcb_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-check &&
                  run pmcb_sum 60 python3 tools/pmc_summary.py gpurun_out/pmcb_fetch/run_counter_collection.csv gpurun_out/pmcb_write/run_counter_collection.csv gpurun_out/pmc_summary.json ;;
        profbench) run profbench 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profbench -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        abmul) for f in ntt-gpu-qtesla_amd/lib/ab/*.so; do b=$(basename $f .so); NTT_AMD_LIB=$PWD/$f run abmul_$b 200 python bench.py --op polymul --steps 5 --warmup 1 --no-cpu-baseline || exit 1; NTT_AMD_LIB=$PWD/$f run abmul1k_$b 200 python bench.py --op polymul --param p-I --steps 5 --warmup 1 --no-cpu-baseline || exit 1; done ;;
        nustest) run nustest 400 python -m pytest tests/test_gpu_nussbaumer.py -x -q -m "gpu and not slow" ;;
        nusbench) run nusbench_q 300 python bench.py --op nussbaumer --ring q --steps 5 --warmup 1 --no-cpu-baseline &&
                  run nusbench_m32 300 python bench.py --op nussbaumer --ring m32 --steps 5 --warmup 1 --no-cpu-baseline &&
                  run nusbench_q1k 300 python bench.py --op nussbaumer --ring q --param p-I --steps 5 --warmup 1 --no-cpu-baseline ;;
        # config 2's launch is ~0.11 ms: 1000 steps (0.1 s) so that the region
        # events time a steady stream of launches, not the clock ramp after idle
        # (20 / 200 / 1000 steps: 0.116 / 0.119 / 0.111 ms, profiles/r03/c2/steps.log)
        # config 1 (one polynomial per call, ~5-8 us of Python submission each) likewise
        bench_c*) c=${step#bench_c}; k=20; [ "$c" = 2 ] || [ "$c" = 1 ] && k=1000; run bench_c$c 500 python bench.py --config $c --steps $k --warmup 3 --cpu-seconds 10 ;;
        # rocprofv3 averages include the warm-up launches (clock ramp): 100 timed
        # steps (config 2: 1000, like its bench line) keep them a small share
        prof_c*) c=${step#prof_c}; k=100; [ "$c" = 2 ] && k=1000; run prof_c$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c$c -o run -- python3 bench.py --config $c --steps $k --warmup 3 --no-cpu-baseline --no-check ;;
        pmc_c*) c=${step#pmc_c}; run pmc_c${c}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c${c}_fetch -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-check &&
                 run pmc_c${c}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c${c}_write -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-check &&
                 run pmc_c${c}_sum 60 python3 tools/pmc_summary.py --config $c --fetch gpurun_out/pmc_c${c}_fetch/run_counter_collection.csv --write gpurun_out/pmc_c${c}_write/run_counter_collection.csv --out gpurun_out/pmc_summary.json ;;
        pmcl_*) n=${step#pmcl_}; b=$((8589934592 / 4 / n)); a="--op fwdinv --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check";
                run pmcl_${n}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcl_${n}_fetch -o run -- python3 bench.py $a &&
                run pmcl_${n}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcl_${n}_write -o run -- python3 bench.py $a &&
                run pmcl_${n}_sum 60 python3 tools/pmc_summary.py --op fwdinv --param p-III-$n --batch $b --fetch gpurun_out/pmcl_${n}_fetch/run_counter_collection.csv --write gpurun_out/pmcl_${n}_write/run_counter_collection.csv --out gpurun_out/pmc_summary.json ;;
        pmcm_*) n=${step#pmcm_}; b=$((1073741824 / n)); a="--op polymul --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check";
                run pmcm_${n}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcm_${n}_fetch -o run -- python3 bench.py $a &&
                run pmcm_${n}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcm_${n}_write -o run -- python3 bench.py $a &&
                run pmcm_${n}_sum 60 python3 tools/pmc_summary.py --op polymul --param p-III-$n --batch $b --fetch gpurun_out/pmcm_${n}_fetch/run_counter_collection.csv --write gpurun_out/pmcm_${n}_write/run_counter_collection.csv --out gpurun_out/pmc_summary.json ;;
        benchm_*) n=${step#benchm_}; b=$((1073741824 / n)); run benchm_$n 300 python bench.py --op polymul --param p-III-$n --batch $b --steps 20 --warmup 3 --cpu-seconds 5 &&
                  run benchmn_$n 300 python bench.py --op polymul_ntt --param p-III-$n --batch $b --steps 20 --warmup 3 --cpu-seconds 5 ;;
        profm_*) n=${step#profm_}; b=$((1073741824 / n)); run profm_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profm_$n -o run -- python3 bench.py --op polymul --param p-III-$n --batch $b --steps 100 --warmup 3 --no-cpu-baseline --no-check ;;
        profl_*) n=${step#profl_}; b=$((8589934592 / 4 / n)); run profl_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profl_$n -o run -- python3 bench.py --op fwdinv --param p-III-$n --batch $b --steps 100 --warmup 3 --no-cpu-baseline --no-check ;;
        benchl_*) n=${step#benchl_}; b=$((8589934592 / 4 / n)); run benchl_$n 300 python bench.py --op fwdinv --param p-III-$n --batch $b --steps 20 --warmup 3 --cpu-seconds 5 ;;
        sq_c*) c=${step#sq_c}; run sq_c$c 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_c$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-check ;;
        sqb_c*) c=${step#sqb_c}; run sqb_c$c 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/sqb_c$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-check ;;
        listpmc) run listpmc 60 rocprofv3 -L ;;
        nusstamps) run nusstamps 200 python tools/nus_stamps.py ntt-gpu-qtesla_amd/lib/diag/nus_stamps*.so ;;
        # round 5: n > 2048 A/B (one process, interleaved) and SQ stall counters
        abl_*) n=${step#abl_}; b=$((8589934592 / 4 / n)); run abl_$n 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-III-$n --batch $b --ops fwd,inv --inplace --rounds 7 ;;
        sql_*) n=${step#sql_}; b=$((8589934592 / 4 / n)); a="--op fwdinv --param p-III-$n --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-check";
               run sql_$n 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sql_$n -o run -- python3 bench.py $a &&
               run sqlb_$n 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/sqlb_$n -o run -- python3 bench.py $a ;;
        # VALU roofline inputs (tools/valu_summary.py): per-opcode issue cost, and
        # SQ_INSTS_VALU + GRBM_GUI_ACTIVE per launch of a config's kernel
        valucost) run valucost 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d gpurun_out/valucost -o run -- ./ntt-gpu-qtesla_amd/bin/valu_cost 16384 ;;
        valum_*) n=${step#valum_}; b=$((1073741824 / n)); run valum_$n 120 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/valum_$n -o run -- python3 bench.py --op polymul --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check ;;
        # round 6: poly_mul_ntt's own FETCH / WRITE and VALU passes and its bench line alone
        pmcmn_*) n=${step#pmcmn_}; b=$((1073741824 / n)); a="--op polymul_ntt --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check";
                 run pmcmn_${n}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcmn_${n}_fetch -o run -- python3 bench.py $a &&
                 run pmcmn_${n}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcmn_${n}_write -o run -- python3 bench.py $a &&
                 run pmcmn_${n}_sum 60 python3 tools/pmc_summary.py --op polymul_ntt --param p-III-$n --batch $b --fetch gpurun_out/pmcmn_${n}_fetch/run_counter_collection.csv --write gpurun_out/pmcmn_${n}_write/run_counter_collection.csv --out gpurun_out/pmc_summary.json ;;
        valumn_*) n=${step#valumn_}; b=$((1073741824 / n)); run valumn_$n 120 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/valumn_$n -o run -- python3 bench.py --op polymul_ntt --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check ;;
        benchmnx_*) n=${step#benchmnx_}; b=$((1073741824 / n)); run benchmn_$n 300 python bench.py --op polymul_ntt --param p-III-$n --batch $b --steps 20 --warmup 3 --cpu-seconds 5 ;;
        valu_c*) c=${step#valu_c}; run valu_c$c 120 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/valu_c$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-check ;;
        # round 6: the small-batch switch per (n, op): latency vs batch kernels
        # from 64 polynomials to the BASELINE batches (tools/switch_sweep.py)
        sweep) run sweep 900 python tools/switch_sweep.py ntt-gpu-qtesla_amd/lib/sweep/a_batch.so ntt-gpu-qtesla_amd/lib/sweep/b_lat.so --out gpurun_out/switch_sweep.json ;;
        sweepfine) run sweepfine 900 python tools/switch_sweep.py ntt-gpu-qtesla_amd/lib/sweep/a_batch.so ntt-gpu-qtesla_amd/lib/sweep/b_lat.so --params ref,p-I,p-III,p-III-4096,p-III-8192 --rounds 7 --refine profiles/r06/sweep/switch_sweep_coarse.json --out gpurun_out/switch_sweep_fine.json ;;
        switchtest) run switchtest 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "latency_switch or golden" --timeout 120 --timeout-method thread ;;
        brtest) run brtest 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -x -q -m gpu -k "bit_reversed or latency_switch or bitrev" --timeout 120 --timeout-method thread ;;
        abbr) run abbr_4096 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so --param p-III-4096 --batch 524288 --ops fwd,fwdbr,inv,invbr --inplace --rounds 7 &&
              run abbr_8192 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so --param p-III-8192 --batch 262144 --ops fwd,fwdbr,inv,invbr --inplace --rounds 7 ;;
        abbr2) run abbr2_4096 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-III-4096 --batch 524288 --ops fwd,fwdbr,inv,invbr --inplace --rounds 7 &&
               run abbr2_8192 300 python tools/ab.py ntt-gpu-qtesla_amd/lib/ab/*.so --param p-III-8192 --batch 262144 --ops fwd,fwdbr,inv,invbr --inplace --rounds 7 ;;
        ab8) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab8/*.so";
             run ab8_p3 300 python tools/ab.py $L --param p-III --batch 1048576 --ops fwd,inv,fwdbr,invbr --rounds 7 &&
             run ab8_p1 300 python tools/ab.py $L --param p-I --batch 1048576 --ops fwd,inv --rounds 7 &&
             run ab8_4096 300 python tools/ab.py $L --param p-III-4096 --batch 524288 --ops fwd,inv --rounds 7 &&
             run ab8_8192 300 python tools/ab.py $L --param p-III-8192 --batch 262144 --ops fwd,inv --rounds 7 ;;
        sweep8) run sweep8 900 python tools/switch_sweep.py ntt-gpu-qtesla_amd/lib/sweep/a_batch.so ntt-gpu-qtesla_amd/lib/sweep/b_lat.so ntt-gpu-qtesla_amd/lib/ab8/lat8.so ntt-gpu-qtesla_amd/lib/ab8/lat16.so --ops fwd,inv,fwdbr,invbr --rounds 5 --out gpurun_out/switch_sweep_latr.json ;;
        floor8) run floor8_p3 300 python tools/latr_floor.py --param p-III &&
                run floor8_p1 300 python tools/latr_floor.py --param p-I ;;
        latsmall) for f in sweep/b_lat ab8/lat8 ab8/lat16; do b=$(basename $f);
                      run latsmall_$b 300 python tools/latency.py --lib ntt-gpu-qtesla_amd/lib/$f.so --batches 1,8,64,256 --params p-I,p-III,p-III-4096,p-III-8192 --rounds 5 || exit 1; done ;;
        ab9) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab9/*.so";
             run ab9_chk 300 python tools/ab.py $L --param p-III --batch 65536 --ops fwd,inv,fwdbr,invbr --rounds 2 &&
             run ab9_p3 300 python tools/ab.py $L --param p-III --batch 1048576 --ops fwd,inv --inplace --rounds 9 &&
             run ab9_p1 300 python tools/ab.py $L --param p-I --batch 1048576 --ops fwd,inv --inplace --rounds 9 ;;
        # round 6: FETCH / WRITE of the one-launch bit-reversed n = 4096 / 8192
        # transforms next to the natural-order ones (same process, ab.py)
        pmcbr) for n in 4096 8192; do b=$((8589934592 / 4 / n)); a="tools/ab.py ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so --param p-III-$n --batch $b --ops fwd,fwdbr,inv,invbr --rounds 1";
                   run pmcbr_${n}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcbr_${n}_fetch -o run -- python3 $a || exit 1;
                   run pmcbr_${n}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcbr_${n}_write -o run -- python3 $a || exit 1; done ;;
        # round 6: rocprofv3 kernel stats of the headline with every transform
        # on the radix-8 / radix-16 one-polynomial-per-workgroup kernels
        proflatr) for v in lat8 lat16; do
                      NTT_AMD_LIB=$PWD/ntt-gpu-qtesla_amd/lib/ab8/$v.so run proflatr_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proflatr_$v -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check || exit 1; done ;;
        ab10) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab10/*.so";
              run ab10_chk 300 python tools/ab.py $L --param p-III --batch 65536 --ops fwd,inv,fwdbr,invbr --rounds 2 &&
              run ab10_chk1 300 python tools/ab.py $L --param p-I --batch 65536 --ops fwd,inv,fwdbr,invbr --rounds 2 &&
              run ab10_p1s 300 python tools/ab.py $L --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 31 &&
              run ab10_p3 300 python tools/ab.py $L --param p-III --batch 1048576 --ops fwd,inv --inplace --rounds 9 &&
              run ab10_p1 300 python tools/ab.py $L --param p-I --batch 1048576 --ops fwd,inv --inplace --rounds 9 &&
              run ab10_4096 300 python tools/ab.py $L --param p-III-4096 --batch 16384 --ops fwd,inv --inplace --rounds 31 &&
              run ab10_8192 300 python tools/ab.py $L --param p-III-8192 --batch 32768 --ops fwd,inv --inplace --rounds 31 ;;
        sweepip) run sweepip 900 python tools/switch_sweep.py ntt-gpu-qtesla_amd/lib/sweep/a_batch.so ntt-gpu-qtesla_amd/lib/sweep/b_lat.so ntt-gpu-qtesla_amd/lib/ab10/r8.so ntt-gpu-qtesla_amd/lib/ab10/r16.so --ops fwd,inv --inplace --rounds 5 --out gpurun_out/switch_sweep_inplace.json ;;
        benchp1) run benchp1 300 python bench.py --op fwdinv --param p-I --batch 1048576 --steps 20 --warmup 3 --no-cpu-baseline ;;
        floorio) run floorio_p1 300 python tools/latr_floor.py --param p-I &&
                 run floorio_p1oop 300 python tools/latr_floor.py --param p-I --oop &&
                 run floorio_p3 300 python tools/latr_floor.py --param p-III &&
                 run floorio_p3oop 300 python tools/latr_floor.py --param p-III --oop ;;
        ab11) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab11/*.so";
              run ab11_chk37 120 python tools/ab.py $L --param p-III-8192 --batch 32805 --ops fwd,inv --rounds 1 &&
              run ab11_chk 300 python tools/ab.py $L --param p-III-8192 --batch 40001 --ops fwd,inv --rounds 2 &&
              run ab11_8192 300 python tools/ab.py $L --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 &&
              run ab11_8192s 300 python tools/ab.py $L --param p-III-8192 --batch 65536 --ops fwd,inv --inplace --rounds 15 ;;
        # round 6: n = 8192 transforms with buffer-resource accesses at 8 / 12 waves
        ab12) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab12/*.so";
              run ab12_chk 300 python tools/ab.py $L --param p-III-8192 --batch 40001 --ops fwd,inv,fwdbr,invbr --rounds 2 &&
              run ab12_8192 300 python tools/ab.py $L --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 &&
              run ab12_8192s 300 python tools/ab.py $L --param p-III-8192 --batch 65536 --ops fwd,inv --inplace --rounds 15 ;;
        # round 6: radix-16 small-batch kernels with the register budget of 7 / 8 waves per SIMD
        ab13) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab13/*.so";
              run ab13_chk 300 python tools/ab.py $L --param p-I --batch 65537 --ops fwd,inv,fwdbr,invbr --rounds 2 &&
              run ab13_c2 300 python tools/ab.py $L --param p-I --batch 65536 --ops fwd,inv --inplace --rounds 31 &&
              run ab13_p1 300 python tools/ab.py $L --param p-I --batch 1048576 --ops fwd,inv --inplace --rounds 9 &&
              run ab13_4096 300 python tools/ab.py $L --param p-III-4096 --batch 16384 --ops fwd,inv --inplace --rounds 31 &&
              run ab13_8192 300 python tools/ab.py $L --param p-III-8192 --batch 32768 --ops fwd,inv --inplace --rounds 31 ;;
        # round 6: software-pipelined n = 4096 / 8192 transforms (BIG_PF)
        ab14) L="ntt-gpu-qtesla_amd/lib/libqtesla_ntt.so ntt-gpu-qtesla_amd/lib/ab14/*.so";
              run ab14_chk8 300 python tools/ab.py $L --param p-III-8192 --batch 40001 --ops fwd,inv --rounds 2 &&
              run ab14_chk4 300 python tools/ab.py $L --param p-III-4096 --batch 40001 --ops fwd,inv --rounds 2 &&
              run ab14_8192 300 python tools/ab.py $L --param p-III-8192 --batch 262144 --ops fwd,inv --inplace --rounds 9 &&
              run ab14_4096 300 python tools/ab.py $L --param p-III-4096 --batch 524288 --ops fwd,inv --inplace --rounds 9 ;;
        sweepbr) run sweepbr 600 python tools/switch_sweep.py ntt-gpu-qtesla_amd/lib/sweep/a_batch.so ntt-gpu-qtesla_amd/lib/sweep/b_lat.so --params p-III-4096,p-III-8192 --ops fwdbr,invbr --out gpurun_out/switch_sweep_br.json ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
