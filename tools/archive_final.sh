#!/bin/bash
# Copy one final-measurement session (tools/gpu_session.sh pytest smoke bench_c*
# benchl_* benchm_* prof_* profl_* profm_* pmc_* pmcl_* pmcm_*) from
# gpurun_out/ into profiles/<dest>/ and make its PMC summary the committed one
# (profiles/pmc_summary.json, read by bench.py).   usage: tools/archive_final.sh r05/final
set -euo pipefail
D=profiles/$1
S=gpurun_out
mkdir -p "$D"
cp $S/session.log $S/smoke.log "$D/"
cp $S/pytest.log "$D/pytest_gpu.log"
for f in $S/bench_c*.log $S/benchl_*.log $S/benchm*.log; do
    python3 - "$f" "$D/$(basename "$f" .log).json" <<'E'
import sys
t = open(sys.argv[1]).read()
i = t.find('{"metric"')
open(sys.argv[2], "w").write(t[i:t.index("\n", i)] + "\n")
E
done
for p in c2 c3 c4 c5; do
    cp $S/prof_$p/run_kernel_stats.csv "$D/rocprof_kernel_stats_$p.csv"
    mkdir -p "$D/pmc_$p"
    cp $S/pmc_${p}_fetch/run_counter_collection.csv "$D/pmc_$p/fetch_counter_collection.csv"
    cp $S/pmc_${p}_write/run_counter_collection.csv "$D/pmc_$p/write_counter_collection.csv"
done
for n in 4096 8192; do
    cp $S/profl_$n/run_kernel_stats.csv "$D/rocprof_kernel_stats_l_$n.csv"
    cp $S/profm_$n/run_kernel_stats.csv "$D/rocprof_kernel_stats_m_$n.csv"
    mkdir -p "$D/pmcmn_$n" "$D/valumn_$n" "$D/valum_$n"
    cp $S/pmcmn_${n}_fetch/run_counter_collection.csv "$D/pmcmn_$n/fetch_counter_collection.csv"
    cp $S/pmcmn_${n}_write/run_counter_collection.csv "$D/pmcmn_$n/write_counter_collection.csv"
    cp $S/valum_$n/run_counter_collection.csv "$D/valum_$n/"
    cp $S/valumn_$n/run_counter_collection.csv "$D/valumn_$n/"
    for k in l m; do
        mkdir -p "$D/pmc${k}_$n"
        cp $S/pmc${k}_${n}_fetch/run_counter_collection.csv "$D/pmc${k}_$n/fetch_counter_collection.csv"
        cp $S/pmc${k}_${n}_write/run_counter_collection.csv "$D/pmc${k}_$n/write_counter_collection.csv"
    done
done
cp $S/pmc_summary.json "$D/"
cp $S/pmc_summary.json profiles/pmc_summary.json
echo "archived into $D"
