set -e
mkdir -p gpurun_out
timeout -k 10 100 python bench.py --op polymul_host --batch 131072 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/host_131072.log 2>&1
timeout -k 10 200 python bench.py --op polymul_host --batch 1048576 --steps 3 --warmup 1 --no-cpu-baseline --chunk 16384 > gpurun_out/host_1M_c16k.log 2>&1
timeout -k 10 100 python - > gpurun_out/pcie_probe.log 2>&1 <<'PY'
import torch, time
x = torch.empty(1<<28, dtype=torch.int32).pin_memory(); d = torch.empty(1<<28, dtype=torch.int32, device='cuda')
for name, f in (("h2d", lambda: d.copy_(x, non_blocking=True)), ("d2h", lambda: x.copy_(d, non_blocking=True))):
    f(); torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(5): f()
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/5
    print(name, 4*(1<<28)/dt/1e9, "GB/s")
PY
