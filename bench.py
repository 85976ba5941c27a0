#!/usr/bin/env python3
"""Benchmark of the north-star path: batched forward + inverse negacyclic NTT,
n = 2048, qTESLA-p-III (q = 856145921), batch = 2^20 polynomials per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

A step = poly_ntt + poly_invntt, in place, over the rank's whole batch (inputs
resident in HBM, generated on the device).  Polynomials are independent, so
the batch shards with no data-path collective: rank r owns polys
[r*B, (r+1)*B) of one global counter-based input stream ("weak" scaling).
torch.distributed (RCCL) is used only for the barrier and the max-over-ranks
time.  Rank 0 prints ONE JSON line.

Roofline: the dominant kernel's average launch duration is measured with HIP
events on the stream the kernels run on; achieved = algorithmic bytes per
launch (8 B per coefficient: one read + one write) / that duration.
cpu_baseline: the oracle's restatement of the reference's serial CPU NTT
(NTT.cu radix2NTT / radix2INTTGS with % q) on this host, rank 0, N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "NTTs/sec (fwd+inv, n=2048 qTESLA-p-III) at batch=2^20; achieved HBM GB/s"
SEED = 0x5EED0003


def shard(total_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak-scaling shard: (first_poly, count) of this rank's slice."""
    return rank * total_per_rank, total_per_rank


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def max_over_ranks(value: float, world: int, device=None) -> float:
    if world <= 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int, device=None):
    if world > 1:
        import torch.distributed as dist
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def cpu_baseline(param: str, seconds: float, threads: int = 1) -> dict:
    """Reference serial CPU NTT restated in the oracle, timed on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    # scale the sample to ~`seconds` of wall time (two refinements: a tiny
    # first sample under-estimates the per-poly time of a multi-thread run)
    count = 8 * threads
    for _ in range(3):
        x = O.fill_uniform(count, param, SEED, 0)
        t = O.time_fwd_inv(x, param, threads, 1)
        if t >= 0.5 * seconds or count >= (1 << 20):
            break
        count = min(max(count, int(count * seconds / max(t, 1e-6))), 1 << 20)
    n = O.params(param)["n"]
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {
        "value": count / t,
        "cpu_model": cpu,
        "nproc": os.cpu_count(),
        "unit": "fwd+inv pairs/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{count} uniform n={n} {param} polys, fwd(Phi twist+bit_reverse_copy+radix2NTT)+"
                  f"inv(radix2INTTGS+bitrev+invPhi) with % q, oracle C restatement of NTT.cu, "
                  f"{threads} thread(s), {t:.1f} s",
    }


def load_pmc(workload: str):
    """HBM traffic per launch from a committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--param", default="p-III")
    ap.add_argument("--batch", type=int, default=1 << 20, help="polynomials per GPU")
    ap.add_argument("--op", default="fwdinv",
                    choices=["fwdinv", "fwd", "inv", "polymul", "polymul_ntt", "nussbaumer", "polymul_host",
                             "fwdinv_host"])
    ap.add_argument("--pageable", action="store_true", help="*_host ops: pageable instead of pinned host buffers")
    ap.add_argument("--chunk", type=int, default=0, help="*_host ops: polys per chunk (0 = library default)")
    ap.add_argument("--slots", type=int, default=0, help="*_host ops: buffer slots (0 = library default)")
    ap.add_argument("--ring", default="q", choices=["q", "m32"], help="--op nussbaumer: mod q or mod 2^32-1")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()

    import torch
    import ntt_amd

    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    if args.op.endswith("_host"):
        return bench_host(args, ntt_amd, torch, device, rank, world)

    pinfo = ntt_amd.param_info(args.param)
    n = pinfo["n"]
    B = args.batch
    first, count = shard(B, rank)
    x = torch.empty(count * n, dtype=torch.int32, device=device)
    ntt_amd.fill_uniform(x, args.param, SEED, first)
    y = z = None
    if args.op in ("polymul", "polymul_ntt", "nussbaumer"):
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        ntt_amd.fill_uniform(y, args.param, SEED ^ 0xFFFF, first)
    stream = torch.cuda.current_stream(device)

    def launch(kind):
        if kind == "fwd":
            ntt_amd.poly_ntt(x, args.param, stream)
        elif kind == "inv":
            ntt_amd.poly_invntt(x, args.param, stream)
        elif kind == "mul":
            ntt_amd.poly_mul(z, x, y, args.param, stream)
        elif kind == "mulntt":
            ntt_amd.poly_mul_ntt(z, x, y, args.param, stream)
        else:
            ntt_amd.poly_mul_nussbaumer(z, x, y, args.param, args.ring, stream)

    kinds = {"fwdinv": ["fwd", "inv"], "fwd": ["fwd"], "inv": ["inv"], "polymul": ["mul"], "polymul_ntt": ["mulntt"],
             "nussbaumer": ["nus"]}[args.op]

    for _ in range(args.warmup):
        for k in kinds:
            launch(k)
    torch.cuda.synchronize(device)

    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in kinds]
           for _ in range(args.steps)]
    barrier(world, device)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s in range(args.steps):
        for i, k in enumerate(kinds):
            evs[s][i][0].record(stream)
            launch(k)
            evs[s][i][1].record(stream)
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    barrier(world, device)
    elapsed = max_over_ranks(t1 - t0, world, device)

    per_kind = {k: sum(evs[s][i][0].elapsed_time(evs[s][i][1]) for s in range(args.steps)) / args.steps
                for i, k in enumerate(kinds)}  # ms per launch
    dom = max(per_kind, key=per_kind.get)
    bytes_per_coeff = 12 if dom in ("mul", "mulntt", "nus") else 8
    alg_bytes = count * n * bytes_per_coeff
    achieved = alg_bytes / (per_kind[dom] * 1e-3) / 1e9

    ok = None
    if not args.no_check:
        if args.op in ("fwdinv",):
            # every step is the identity: the buffer must equal the regenerated input
            ref = torch.empty_like(x)
            ntt_amd.fill_uniform(ref, args.param, SEED, first)
            ok = bool(torch.equal(ref, x))
            del ref
        ok = bool(max_over_ranks(0.0 if ok in (None, True) else 1.0, world, device) == 0.0) if ok is not None else None

    units = world * count * args.steps
    value = units / elapsed
    workload = {"fwdinv": "fwd+inv negacyclic NTT", "fwd": "forward negacyclic NTT",
                "inv": "inverse negacyclic NTT", "polymul": "fused negacyclic poly-mul",
                "polymul_ntt": "fused negacyclic poly-mul, second operand in the NTT domain",
                "nussbaumer": "Nussbaumer negacyclic product" + (" mod 2^32-1" if args.ring == "m32" else "")}[args.op]
    workload = f"{workload} n={n} qTESLA-{args.param}" if args.param != "ref" else f"{workload} n={n} ref q={pinfo['q']}"
    unit = {"fwdinv": "fwd+inv pairs/s", "fwd": "NTTs/s", "inv": "INTTs/s", "polymul": "products/s",
            "polymul_ntt": "products/s",
            "nussbaumer": "products/s"}[args.op]
    out = {
        "metric": METRIC if args.op == "fwdinv" and args.param == "p-III" else f"{unit} ({workload})",
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device counter-based uniform coefficients in [0,q))",
        "config": {"workload": workload, "param_set": args.param, "n": n, "q": pinfo["q"],
                   "batch_per_gpu": count, "global_batch": world * count, "parallelism": f"batch-shard x{world}"},
        "hbm_gbs_algorithmic": value * n * (bytes_per_coeff if args.op != "fwdinv" else 16) / 1e9,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_pmc(workload),
                     "avg_launch_ms": per_kind[dom], "alg_bytes_per_launch": alg_bytes,
                     "per_kernel_ms": per_kind},
        "check": {"roundtrip_identity_full_batch": ok},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.param, args.cpu_seconds, 1)
        # the same restatement batch-parallel over this box's CPU share
        threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        out["cpu_baseline_all_cores"] = cpu_baseline(args.param, args.cpu_seconds / 2, threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if ok is False:
        sys.exit(1)


def bench_host(args, ntt_amd, torch, device, rank, world):
    """Host -> host operation through ntt_host_ctx: the
    reference's PCIe-inclusive timing (NTT.cu:2384-2428), pipelined.  Never
    the headline `value` of the device-resident metric."""
    import numpy as np
    pinfo = ntt_amd.param_info(args.param)
    n = pinfo["n"]
    B = args.batch
    first, count = shard(B, rank)
    nin = 2 if args.op == "polymul_host" else 1

    def host_buf(seed):
        t = torch.empty(count * n, dtype=torch.int32, device=device)
        if seed is not None:
            ntt_amd.fill_uniform(t, args.param, seed, first)
        arr = np.empty((count, n), np.uint32) if args.pageable else ntt_amd.host_empty(count * n).reshape(count, n)
        arr[...] = t.cpu().numpy().view(np.uint32).reshape(count, n)
        return arr

    a = host_buf(SEED)
    b = host_buf(SEED ^ 0xFFFF) if nin == 2 else None
    c = host_buf(None)
    ctx = ntt_amd.HostContext(args.param, args.chunk, args.slots)

    def step():
        if nin == 2:
            ctx.mul(c, a, b)
        else:
            ctx.ntt(c, a)
            ctx.invntt(c, c)

    for _ in range(args.warmup):
        step()
    barrier(world, device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    barrier(world, device)
    elapsed = max_over_ranks(t1 - t0, world, device)
    ok = None
    if not args.no_check:
        ok = bool(np.array_equal(c, a)) if nin == 1 else None
    ctx.close()
    units = world * count * args.steps
    value = units / elapsed
    # PCIe bytes per unit: polymul 2 in + 1 out; fwd+inv 2 in + 2 out
    pcie_bytes = (3 if nin == 2 else 4) * n * 4
    workload = ("host->host fused negacyclic poly-mul" if nin == 2 else "host->host fwd+inv negacyclic NTT") + \
        f" n={n} qTESLA-{args.param} ({'pageable' if args.pageable else 'pinned'} buffers, PCIe in the timed region)"
    out = {
        "metric": f"{'products/s' if nin == 2 else 'fwd+inv pairs/s'} ({workload})",
        "value": value, "unit": "products/s" if nin == 2 else "fwd+inv pairs/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic (device counter-based uniform coefficients in [0,q))",
        "config": {"workload": workload, "param_set": args.param, "n": n, "batch_per_gpu": count,
                   "chunk_polys": args.chunk or 4096, "slots": args.slots or 3,
                   "global_batch": world * count, "parallelism": f"batch-shard x{world}"},
        "pcie_gbs": value * pcie_bytes / 1e9 / world,
        "check": {"roundtrip_identity_full_batch": ok},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
