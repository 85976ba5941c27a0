set -e
for cs in "1024 3" "4096 2" "4096 3" "4096 4" "16384 3" "8192 4"; do
  set -- $cs
  timeout -k 10 100 python bench.py --op polymul_host --batch 131072 --steps 3 --warmup 1 --chunk $1 --slots $2 > gpurun_out/sw_$1_$2.log 2>&1
done
python - <<'PY'
import torch, time
x = torch.empty(1<<28, dtype=torch.int32).pin_memory(); d = torch.empty(1<<28, dtype=torch.int32, device='cuda')
for name, f in (("h2d", lambda: d.copy_(x, non_blocking=True)), ("d2h", lambda: x.copy_(d, non_blocking=True))):
    f(); torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(5): f()
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/5
    print(name, 4*(1<<28)/dt/1e9, "GB/s")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream(); y = torch.empty_like(x).pin_memory(); d2 = torch.empty_like(d)
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(5):
    with torch.cuda.stream(s1): d.copy_(x, non_blocking=True)
    with torch.cuda.stream(s2): y.copy_(d2, non_blocking=True)
torch.cuda.synchronize(); dt=(time.perf_counter()-t)/5
print("duplex", 2*4*(1<<28)/dt/1e9, "GB/s total")
PY
