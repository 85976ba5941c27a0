set -e
mkdir -p gpurun_out
for n in 4096 8192; do
  b=$((1073741824 / 4 / n * 2)); b=$((2147483648 / 4 / n))
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/lpmc_${n}_f -o run -- python3 bench.py --op fwdinv --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/lpmc_${n}_f.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/lpmc_${n}_w -o run -- python3 bench.py --op fwdinv --param p-III-$n --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/lpmc_${n}_w.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lpmc_${n}_sq -o run -- python3 bench.py --op fwdinv --param p-III-$n --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/lpmc_${n}_sq.log 2>&1
done
