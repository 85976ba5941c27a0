#!/usr/bin/env python3
"""Benchmark of the north-star path: batched forward + inverse negacyclic NTT,
n = 2048, qTESLA-p-III (q = 856145921), batch = 2^20 polynomials per GPU
(BASELINE.json config 3, the default), and the other BASELINE configs:

    python bench.py [--gpus N] [--steps K] [--warmup W]          # config 3
    python bench.py --config {1,2,3,4,5} ...                      # BASELINE configs
    torchrun --nproc-per-node N bench.py --gpus N ...             # one rank per GPU

--gpus N > 1 without a launcher (no WORLD_SIZE in the environment): the
process starts N fresh child ranks itself before it touches the GPU
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set),
relays rank 0's JSON line and exits with the worst child status.  Every rank
needs a device of its own: fewer visible devices than ranks is an error
unless --allow-shared-devices (the world-size-2 rehearsal on a one-GPU box).

  config 1  single forward NTT n=1024 p-I: the reference's serial CPU path
            (plumbing); the GPU line is the batch-1 launch latency
  config 2  forward NTT n=1024 p-I, batch 65536
  config 3  forward + inverse NTT n=2048 p-III, batch 2^20 (headline)
  config 4  fused negacyclic poly-mul n=2048 p-III, 2^20 per GPU (2^23 on 8)
  config 5  Nussbaumer negacyclic product n=2048 p-III, 2^20 (mod q)

A step = one pass of the configured operation over the rank's whole batch
(inputs resident in HBM, generated on the device; the transforms in place,
as the reference's kernels).  Polynomials are independent, so the batch
shards with no data-path collective: rank r owns polys [r*B, (r+1)*B) of one
global counter-based input stream ("weak" scaling).  torch.distributed
(gloo by default: CPU tensors, no GPU collective on the path; RCCL with
--dist-backend nccl) is used only for the barrier and the max / min over
ranks of the timed region.  Rank 0 prints ONE JSON line.

Roofline: the dominant kernel's average launch duration is measured with HIP
events on the stream the kernels run on; achieved = algorithmic bytes per
launch (8 B per coefficient for a transform, 12 B for a product) / that
duration.  traffic = measured HBM bytes per launch from
profiles/pmc_summary.json, only when it was taken on this library build.

After the timed region, outside it (the checker legs, like cpu_baseline):
the transform round trip over the whole batch on device, and >= 64 sampled
polynomials of one more launch on the regenerated input compared with the
CPU oracle (oracle/, test infrastructure; never the measured path).
cpu_baseline: the oracle's restatement of the reference's serial CPU path
for the same operation, on this host, rank 0 at N = 1 only.
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
PEAK_CLOCK_GHZ = 2.4         # MI355X peak engine clock
SIMDS_PER_CU = 4
# ops whose dominant kernel is bound by VALU issue, not HBM:
# their line's roofline is the VALU one, the HBM fraction a secondary field
VALU_BOUND = {"polymul", "polymul_ntt", "nussbaumer"}
METRIC = "NTTs/sec (fwd+inv, n=2048 qTESLA-p-III) at batch=2^20; achieved HBM GB/s"
SEED = 0x5EED0003
PMC_PATH = os.path.join(ROOT, "profiles", "pmc_summary.json")
# tools-only diagnostic library (ntt-gpu-qtesla_amd/tools/ntt_diag.hip, `make tools`):
# the transforms' memory-only variants for roofline.pattern_floor_ms
DIAG_PATH = os.path.join(ROOT, "ntt-gpu-qtesla_amd", "lib", "libqtesla_ntt_diag.so")
# the library's small-batch switch entry points of each bench op
# (ntt_small_batch_max, csrc/ntt_lat.hpp: one threshold per (n, op))
SWITCH_OPS = {"fwd": ["fwd"], "inv": ["inv"], "fwdinv": ["fwd", "inv"], "polymul": ["mul"],
              "polymul_ntt": ["mul_ntt"], "nussbaumer": []}


def runs_latency_kernels(ntt_amd, op: str, param: str, batch: int) -> bool:
    """True when some launch of a step of `op` at `batch` polynomials runs
    the small-batch kernels (one polynomial per workgroup, csrc/ntt_lat.hpp)."""
    return any(batch <= ntt_amd.small_batch_max(param, k) for k in SWITCH_OPS[op])

# BASELINE.json configs -> (op, param, batch per GPU, ring)
CONFIGS = {
    1: ("fwd", "p-I", 1, "q"),
    2: ("fwd", "p-I", 65536, "q"),
    3: ("fwdinv", "p-III", 1 << 20, "q"),
    4: ("polymul", "p-III", 1 << 20, "q"),
    5: ("nussbaumer", "p-III", 1 << 20, "q"),
}
OPS = ["fwdinv", "fwd", "inv", "polymul", "polymul_ntt", "nussbaumer", "polymul_host", "fwdinv_host"]
UNIT = {"fwdinv": "fwd+inv pairs/s", "fwd": "NTTs/s", "inv": "INTTs/s", "polymul": "products/s",
        "polymul_ntt": "products/s", "nussbaumer": "products/s"}


def shard(total_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak-scaling shard: (first_poly, count) of this rank's slice."""
    return rank * total_per_rank, total_per_rank


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nranks: int, argv: list[str]) -> int:
    """Launcher-free multi-GPU run: start `nranks` fresh child processes of
    this script, one per GPU, with the torch.distributed env set.  Called
    before this process makes any GPU call (it never initialises HIP: the
    children do).  Rank 0 inherits stdout and prints the one JSON line; if a
    rank fails, the others are stopped (by PID) and the worst status is
    returned."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(nranks):
        env = {**os.environ, "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nranks),
               "LOCAL_WORLD_SIZE": str(nranks), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
               "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")}
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    worst = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                worst = worst or rc
                for o in live:          # a failed rank would leave the others waiting in a barrier
                    o.terminate()
        if live:
            time.sleep(0.05)
    return worst if worst >= 0 else 128 - worst


def check_devices(world: int, allow_shared: bool) -> int | None:
    """One device per rank, or exit status 3 with the reason (unless shared
    devices were asked for).  Counting devices does not initialise HIP."""
    import torch
    ndev = torch.cuda.device_count()
    if ndev < 1:
        print("error: no GPU visible (the product has no CPU path)", file=sys.stderr)
        return 3
    if ndev < world and not allow_shared:
        print(f"error: {world} ranks but only {ndev} visible device(s); every rank needs its own GPU "
              f"(--allow-shared-devices runs ranks on shared devices, for rehearsals only)", file=sys.stderr)
        return 3
    return None


class Dist:
    """The only collectives of the bench: barrier and max over ranks."""

    def __init__(self, world: int, backend: str, device):
        self.world, self.backend, self.device = world, backend, device
        if world > 1:
            import torch.distributed as dist
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group("gloo")

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def _reduce(self, value: float, op: str) -> float:
        if self.world <= 1:
            return value
        import torch
        import torch.distributed as dist
        t = torch.tensor([value], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
        return float(t.item())

    def max(self, value: float) -> float:
        return self._reduce(value, "max")

    def min(self, value: float) -> float:
        return self._reduce(value, "min")

    def close(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        return "unknown"


def cpu_baseline(op: str, param: str, seconds: float, threads: int = 1, ring: str = "q", max_count=1 << 20) -> dict:
    """The reference's serial CPU path for `op`, restated in the oracle, timed
    on a bounded sample of the workload (about `seconds` of wall time)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    top = {"fwdinv": "fwdinv", "fwd": "fwd", "inv": "inv", "polymul": "polymul", "polymul_ntt": "polymul",
           "nussbaumer": "nussbaumer_m32" if ring == "m32" else "nussbaumer_q"}[op]
    count = 8 * threads
    for _ in range(4):   # scale the sample to ~`seconds` (a tiny first sample under-estimates)
        x = O.fill_uniform(count, param, SEED, 0)
        y = O.fill_uniform(count, param, SEED ^ 0xFFFF, 0)
        t = O.time_op(top, x, param, threads, 1, y=y)
        if t >= 0.5 * seconds or count >= max_count:
            break
        count = min(max(count + 1, int(count * seconds / max(t, 1e-6))), max_count)
    n = O.params(param)["n"]
    what = {"fwdinv": "fwd (Phi twist + bit_reverse_copy + radix2NTT) + inv (radix2INTTGS + bitrev + invPhi)",
            "fwd": "fwd (Phi twist + bit_reverse_copy + radix2NTT, NTT.cu:1908-1926)",
            "inv": "inv (radix2INTTGS + bitrev + invPhi)",
            "polymul": "test_NTT_nega_CT composition: fwd(a), fwd(b), pointwise, inv (NTT.cu:1908-1946)",
            "nussbaumer_m32": "nussbaumer_fft mod 2^32-1 (NTT.cu:167-277), m=32",
            "nussbaumer_q": "nussbaumer_fft's algorithm mod q (NTT.cu:167-277), m=32"}[top]
    return {
        "value": count / t,
        "unit": UNIT.get(op, "units/s"),
        "cores": threads,
        "kind": "port",
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
        "sample": f"{count} uniform n={n} {param} polys: {what}{'' if top == 'nussbaumer_m32' else ' with % q'}, "
                  f"oracle C restatement of NTT.cu, "
                  f"{threads} thread(s), {t:.2f} s",
    }


def load_pmc(workload: str, batch: int, build_hash: str):
    """HBM traffic per launch from the committed rocprofv3 PMC summary, only
    when it was measured on this exact library build (else None + why)."""
    try:
        with open(PMC_PATH) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_summary.json"
    e = d.get("entries", {}).get(workload)
    if e is None:
        return None, "no PMC entry for this workload"
    if e.get("batch") != batch:
        return None, f"PMC entry measured at batch {e.get('batch')}"
    if e.get("build_hash") != build_hash:
        return None, f"PMC entry measured on build {e.get('build_hash')}, this library is {build_hash}"
    return e.get("hbm_bytes_per_launch"), "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, this build"


def load_valu(workload: str, batch: int, build_hash: str, kernel_key: str):
    """VALU issue demand per launch of the dominant kernel (SIMD-cycles, from
    SQ_INSTS_VALU x the kernel's opcode mix weighted by the measured issue
    costs, tools/valu_summary.py), only when measured on this build."""
    try:
        with open(PMC_PATH) as f:
            e = json.load(f).get("entries", {}).get(workload)
    except (OSError, ValueError):
        return None, "no profiles/pmc_summary.json"
    if e is None or "valu" not in e:
        return None, "no VALU counter entry for this workload"
    if e.get("batch") != batch:
        return None, f"VALU entry measured at batch {e.get('batch')}"
    if e.get("build_hash") != build_hash:
        return None, f"VALU entry measured on build {e.get('build_hash')}, this library is {build_hash}"
    k = e["valu"]["kernels"].get(kernel_key)
    if k is None:
        return None, f"no VALU entry for kernel {kernel_key}"
    return dict(k, cus=e["valu"].get("cus", 256)), "rocprofv3 SQ_INSTS_VALU x opcode-mix issue cost, this build"


def valu_roofline(v, launch_ms: float, hbm: dict) -> dict:
    """achieved = VALU issue SIMD-cycles per launch / live launch time;
    peak = 4 SIMDs x CUs x 2.4 GHz (frac).  frac_at_held_clock is taken from
    the counter pass ALONE: its VALU SIMD-cycles over its own cycles
    (GRBM_GUI_ACTIVE / 8 XCDs) for the same dispatches, i.e. how busy the
    VALU was at the clock the chip held -- never the counter pass's cycles
    over this run's (faster, unprofiled) launch time."""
    if v is None:
        return {"bound": "valu", "achieved": None, "peak": None, "unit": "G SIMD-cycles/s", "frac": None, "hbm": hbm}
    cyc = v["valu_simd_cycles_per_launch"]
    achieved = cyc / (launch_ms * 1e-3) / 1e9
    peak = SIMDS_PER_CU * v["cus"] * PEAK_CLOCK_GHZ
    held = v.get("valu_busy_at_pmc_clock")
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "G SIMD-cycles/s", "frac": achieved / peak,
            "frac_at_held_clock": held, "clock_ghz_pmc": v.get("clock_ghz_pmc"),
            "held_clock_source": "counter pass: VALU SIMD-cycles / (4 SIMDs x CUs x GRBM_GUI_ACTIVE/8), same dispatches"
            if held is not None else "not in this PMC entry (written before the field existed)",
            "valu_insts_per_launch": v["SQ_INSTS_VALU"], "mean_simd_cycles_per_valu": v["mean_simd_cycles_per_valu"],
            "valu_simd_cycles_per_launch": cyc, "uncosted_opcodes": v.get("uncosted_opcodes"), "hbm": hbm}


def pattern_floor(args, ntt_amd, torch, x, stream, steps: int):
    """The memory-only variant of the dominant transform kernels: the same
    grid, loads, LDS exchanges / transposes and stores, no arithmetic, of the
    kernel family the line's launches run (tools-only diagnostic library,
    tools/ntt_diag.hip: ntt_debug_variant op 0/1 variant 3 for the batch
    kernels, op 5/6 variant 1/5 for the radix-8/16 one-polynomial-per-workgroup
    kernels, op 7 variant 1/3 for the n = 4096 / 8192 one-wave kernels), timed
    in this process AFTER the timed region on the same buffer
    (its contents no longer matter), with an event pair around `steps`
    back-to-back launches on the kernels' stream.  It is the access pattern's
    own floor: kernel / floor says how much the arithmetic costs the memory
    stream.  Never part of `value`."""
    import ctypes
    if args.op not in ("fwdinv", "fwd", "inv"):
        return None
    if not os.path.exists(DIAG_PATH):
        return {"note": f"{os.path.relpath(DIAG_PATH, ROOT)} not built (make -C ntt-gpu-qtesla_amd tools)"}
    npoly = x.numel() // ntt_amd.param_info(args.param)["n"]
    kinds = {"fwdinv": ["fwd", "inv"], "fwd": ["fwd"], "inv": ["inv"]}[args.op]
    variants = {}
    for k in kinds:
        radix = ntt_amd.small_batch_radix(args.param, k, npoly)
        if radix == 0 and ntt_amd.param_info(args.param)["n"] > 2048:
            variants[k] = (7, 1 if k == "fwd" else 3,
                           f"k_big_mem<PS, {'false' if k == 'fwd' else 'true'}> (loads + chunk LDS transposes + stores)")
        elif radix == 0:
            variants[k] = (0 if k == "fwd" else 1, 3, "k_variant<PS, INV, 3> (loads + LDS transpose + stores)")
        elif radix in (8, 16):
            variants[k] = (5 if radix == 8 else 6, 1 if k == "fwd" else 5,
                           f"k_ntt_latr<PS, INV, false, {3 if radix == 8 else 4}, 1> (loads + LDS exchanges + stores)")
        else:
            return {"note": "small batch: the radix-4 latency kernels (csrc/ntt_lat.hpp) run it; "
                            "the diagnostic library has no memory-only variant of them"}
    L = ctypes.CDLL(DIAG_PATH)
    vp = ctypes.c_void_p
    L.ntt_debug_variant.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    ps = ntt_amd.PARAM_SETS[args.param]
    sp = vp(stream.cuda_stream)
    ms = {}
    for k in kinds:
        op, var, _ = variants[k]

        def run():
            rc = L.ntt_debug_variant(op, var, vp(x.data_ptr()), vp(x.data_ptr()), npoly, ps, sp)
            if rc != 0:
                raise RuntimeError(f"ntt_debug_variant({op}, {var}) failed: {rc}")
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(x.device)
        e0.record(stream)
        for _ in range(steps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(x.device)
        ms[k] = e0.elapsed_time(e1) / steps
    return {"ms": ms, "steps": steps,
            "kernel": {k: v[2] + ", no arithmetic (tools/ntt_diag.hip)" for k, v in variants.items()},
            "timing": "region events / steps, after the timed region"}


def workload_name(op, param, n, q, ring):
    base = {"fwdinv": "fwd+inv negacyclic NTT", "fwd": "forward negacyclic NTT", "inv": "inverse negacyclic NTT",
            "polymul": "fused negacyclic poly-mul",
            "polymul_ntt": "fused negacyclic poly-mul, second operand in the NTT domain",
            "nussbaumer": "Nussbaumer negacyclic product" + (" mod 2^32-1" if ring == "m32" else "")}[op]
    return f"{base} n={n} qTESLA-{param}" if param != "ref" else f"{base} n={n} ref q={q}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                    help="BASELINE.json config (sets op / param / batch defaults)")
    ap.add_argument("--op", default=None, choices=OPS)
    ap.add_argument("--param", default=None, choices=["ref", "p-I", "p-III", "p-III-4096", "p-III-8192"],
                    help="p-III-4096 / p-III-8192: the n > 2048 four-step transforms (fwd / inv / fwdinv only)")
    ap.add_argument("--batch", type=int, default=None, help="polynomials per GPU")
    ap.add_argument("--ring", default=None, choices=["q", "m32"], help="--op nussbaumer: mod q or mod 2^32-1")
    ap.add_argument("--allow-shared-devices", action="store_true",
                    help="let ranks share devices when fewer than --gpus are visible (one-GPU rehearsals only)")
    ap.add_argument("--dist-backend", default="gloo", choices=["gloo", "nccl"],
                    help="process group for the barrier / max-over-ranks only (no data-path collective, so "
                         "gloo on CPU tensors by default; nccl = RCCL)")
    ap.add_argument("--pageable", action="store_true", help="*_host ops: pageable instead of pinned host buffers")
    ap.add_argument("--chunk", type=int, default=0, help="*_host ops: polys per chunk (0 = library default)")
    ap.add_argument("--slots", type=int, default=0, help="*_host ops: buffer slots (0 = library default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--no-floor", action="store_true", help="skip roofline.pattern_floor_ms (transforms)")
    args = ap.parse_args()
    c_op, c_param, c_batch, c_ring = CONFIGS[args.config]
    args.op = args.op or c_op
    args.param = args.param or c_param
    args.batch = args.batch or c_batch
    args.ring = args.ring or c_ring

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    rc = check_devices(world, args.allow_shared_devices)
    if rc is not None:
        sys.exit(rc)

    import torch
    import ntt_amd

    # one rank per GPU; with --allow-shared-devices ranks beyond the visible
    # devices share them (the world-size-2 rehearsal on a one-GPU box)
    dev_index = local % torch.cuda.device_count()
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    dist = Dist(world, args.dist_backend, device)

    if args.op.endswith("_host"):
        return bench_host(args, ntt_amd, torch, device, rank, world, dist)

    pinfo = ntt_amd.param_info(args.param)
    n = pinfo["n"]
    first, count = shard(args.batch, rank)
    x = torch.empty(count * n, dtype=torch.int32, device=device)
    ntt_amd.fill_uniform(x, args.param, SEED, first)
    y = z = None
    if args.op in ("polymul", "polymul_ntt", "nussbaumer"):
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        ntt_amd.fill_uniform(y, args.param, SEED ^ 0xFFFF, first)
    stream = torch.cuda.current_stream(device)

    def launch(kind, st=stream):
        if kind == "fwd":
            ntt_amd.poly_ntt(x, args.param, st)
        elif kind == "inv":
            ntt_amd.poly_invntt(x, args.param, st)
        elif kind == "mul":
            ntt_amd.poly_mul(z, x, y, args.param, st)
        elif kind == "mulntt":
            ntt_amd.poly_mul_ntt(z, x, y, args.param, st)
        else:
            ntt_amd.poly_mul_nussbaumer(z, x, y, args.param, args.ring, st)

    kinds = {"fwdinv": ["fwd", "inv"], "fwd": ["fwd"], "inv": ["inv"], "polymul": ["mul"], "polymul_ntt": ["mulntt"],
             "nussbaumer": ["nus"]}[args.op]

    for _ in range(args.warmup):
        for k in kinds:
            launch(k)
    torch.cuda.synchronize(device)

    # Kernel durations from HIP events on the launch stream.  With several
    # kinds per step (fwd + inv) every launch has its own event pair; with one
    # kind the pair brackets the whole timed region and the average is
    # region / steps: per-launch event pairs add ~5 us to a ~0.1 ms launch
    # (config 2: 117.8 us per-launch events vs rocprofv3 111.8 us).
    single = len(kinds) == 1
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in kinds]
           for _ in range(1 if single else args.steps)]
    dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    if single:
        evs[0][0][0].record(stream)
    for s in range(args.steps):
        for i, k in enumerate(kinds):
            if not single:
                evs[s][i][0].record(stream)
            launch(k)
            if not single:
                evs[s][i][1].record(stream)
    if single:
        evs[0][0][1].record(stream)
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    dist.barrier()
    elapsed = dist.max(t1 - t0)
    fastest = dist.min(t1 - t0)

    median_kind = None   # one event pair around the region: no per-launch spread
    if single:
        per_kind = {kinds[0]: evs[0][0][0].elapsed_time(evs[0][0][1]) / args.steps}
    else:
        per_kind = {k: sum(evs[s][i][0].elapsed_time(evs[s][i][1]) for s in range(args.steps)) / args.steps
                    for i, k in enumerate(kinds)}  # ms per launch
        import statistics
        median_kind = {k: statistics.median(evs[s][i][0].elapsed_time(evs[s][i][1]) for s in range(args.steps))
                       for i, k in enumerate(kinds)}
    dom = max(per_kind, key=per_kind.get)
    bytes_per_coeff = 12 if dom in ("mul", "mulntt", "nus") else 8
    alg_bytes = count * n * bytes_per_coeff
    achieved = alg_bytes / (per_kind[dom] * 1e-3) / 1e9

    check = {"roundtrip_identity_full_batch": None, "sampled_vs_oracle": None}
    if not args.no_check:
        check = checker_legs(args, ntt_amd, torch, x, y, z, first, count, n)
    expiries = None
    if ntt_amd.param_info(args.param)["n"] > 2048:
        # the n > 2048 kernels' slot barriers: an expired wait poisons its
        # polynomial (sentinel output) and counts here, read after the timed
        # region AND the checker legs' own launches; any count fails the run
        torch.cuda.synchronize(device)
        expiries = ntt_amd.sync_expiries()
    if not args.no_check:
        bad = 0.0 if all(v is None or v is True or (isinstance(v, dict) and v.get("ok")) for v in check.values()) \
            else 1.0
        if expiries:
            bad = 1.0
        check["all_ranks_ok"] = dist.max(bad) == 0.0
    if expiries is not None:
        check["slot_sync_expiries"] = expiries
    latency = None
    if runs_latency_kernels(ntt_amd, args.op, args.param, count) and n <= 2048:
        try:   # beside the line, like the floor: never part of `value`
            latency = graph_replay(torch, launch, kinds, max(args.steps, 50), device)
        except Exception as e:   # noqa: BLE001
            latency = {"note": f"graph replay not measured: {type(e).__name__}: {e}"}
        latency["api_us_per_step"] = None   # filled in below from the timed region
    floor = None
    if not args.no_floor:
        try:   # a diagnostic beside the line: it must never cost the measurement itself
            floor = pattern_floor(args, ntt_amd, torch, x, stream, max(args.steps, 10))
        except Exception as e:   # noqa: BLE001
            floor = {"note": f"pattern floor not measured: {type(e).__name__}: {e}"}

    units = world * count * args.steps
    value = units / elapsed
    workload = workload_name(args.op, args.param, n, pinfo["q"], args.ring)
    unit = UNIT[args.op]
    build_hash = ntt_amd.build_hash()
    traffic, traffic_note = load_pmc(workload, count, build_hash)
    hbm = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_note": traffic_note,
           "avg_launch_ms": per_kind[dom], "alg_bytes_per_launch": alg_bytes,
           "timing": "region events / steps" if single else "per-launch events", "per_kernel_ms": per_kind}
    if median_kind is not None:
        hbm["per_kernel_median_ms"] = median_kind
    if floor is not None:
        hbm["pattern_floor"] = floor
        if dom in floor.get("ms", {}):
            hbm["pattern_floor_ms"] = floor["ms"][dom]
            hbm["kernel_over_floor"] = per_kind[dom] / floor["ms"][dom]
            hbm["floor_frac"] = alg_bytes / (floor["ms"][dom] * 1e-3) / 1e9 / HBM_PEAK_GBS
    if args.op in VALU_BOUND:
        v, v_note = load_valu(workload, count, build_hash, dom)
        roofline = dict(valu_roofline(v, per_kind[dom], hbm), kernel=dom, valu_note=v_note,
                        avg_launch_ms=per_kind[dom], per_kernel_ms=per_kind)
    else:
        roofline = hbm
    if latency is not None:
        latency["api_us_per_step"] = elapsed / args.steps * 1e6
        if rank == 0 and world == 1 and args.op in ("fwd", "inv", "polymul"):
            latency.update(native_latency(args, count))
        roofline["latency"] = latency
    headline = args.op == "fwdinv" and args.param == "p-III" and args.batch == 1 << 20
    out = {
        "metric": METRIC if headline else f"{unit} ({workload}, batch {args.batch} per GPU)",
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "rank_ms_per_step": {"max": elapsed / args.steps * 1e3, "min": fastest / args.steps * 1e3},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device counter-based uniform coefficients in [0,q))",
        "config": {"workload": workload, "baseline_config": args.config if (args.op, args.param, args.batch) ==
                   CONFIGS[args.config][:3] else None, "param_set": args.param, "n": n, "q": pinfo["q"],
                   "batch_per_gpu": count, "global_batch": world * count, "parallelism": f"batch-shard x{world}",
                   "dist_backend": args.dist_backend if world > 1 else None},
        "hbm_gbs_algorithmic": value * n * (bytes_per_coeff if args.op != "fwdinv" else 16) / 1e9,
        # a fwd+inv pair is two transforms; stated to remove the ambiguity
        "transforms_per_s": 2 * value if args.op == "fwdinv" else None,
        "roofline": roofline,
        "check": check,
        "build": {"hash": build_hash},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out.update(cpu_baseline_legs(args, n))
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()
    if (not args.no_check and not check.get("all_ranks_ok", True)) or expiries:
        sys.exit(1)


def graph_replay(torch, launch, kinds, steps, device):
    """Small batches are latency-bound: the timed region's rate is the Python
    -> C ABI submission cost, not the GPU's.  Here `steps` steps are captured
    once in a HIP graph (torch.cuda.CUDAGraph; the library's launches go to
    the capturing stream) and replayed with an event pair around the replay:
    the GPU time per step without host submission (kernel + launch boundary),
    what a C caller's back-to-back loop approaches (ntt_main -speedgpu 12).
    Never part of `value`."""
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.graph(g, stream=side):
        for _ in range(steps):
            for k in kinds:
                launch(k, side)
    g.replay()   # warm
    torch.cuda.synchronize(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(device)
    e0.record(cur)
    g.replay()
    e1.record(cur)
    torch.cuda.synchronize(device)
    return {"graph_replay_us_per_step": e0.elapsed_time(e1) * 1e3 / steps, "graph_steps": steps,
            "kernels": "small-batch kernels, one polynomial per n/4-thread workgroup (csrc/ntt_lat.hpp)"}


def native_latency(args, batch):
    """The same calls from C++ through the C ABI, back to back on one stream
    (`ntt_main -speedgpu 12`, a child process): what the qTESLA signing loop,
    a C program, pays per call without Python's submission cost.  Beside the
    line, never part of `value`; a failure is reported, not raised."""
    import subprocess
    exe = os.path.join(ROOT, "ntt-gpu-qtesla_amd", "bin", "ntt_main")
    op = {"fwd": "poly_ntt", "inv": "poly_invntt", "polymul": "poly_mul"}[args.op]
    try:
        r = subprocess.run([exe, "-speedgpu", "12", "-param", args.param, "-batch", str(batch), "-reps", "2000"],
                           capture_output=True, text=True, timeout=120)
        for line in r.stdout.splitlines():
            if line.startswith("{") and json.loads(line).get("op") == op:
                d = json.loads(line)
                return {"native_c_abi_us_per_call": d["back_to_back_us"],
                        "native_round_trip_us": d["round_trip_us"],
                        "native_note": "ntt_main -speedgpu 12: 2000 calls back to back on one stream "
                                       "(round trip: a stream synchronisation after every call)"}
        return {"native_note": f"ntt_main -speedgpu 12 gave no {op} line (rc {r.returncode})"}
    except Exception as e:   # noqa: BLE001
        return {"native_note": f"ntt_main -speedgpu 12 not run: {type(e).__name__}: {e}"}


def host_threads():
    """Threads for the batch-parallel CPU leg and why: the box's CPU share
    (OMP_NUM_THREADS, which the GPU pool sets to the share of one GPU),
    else the CPUs this process may run on."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env), visible, f"OMP_NUM_THREADS={env} (this box's CPU share per GPU); {visible} CPUs visible"
    return visible, visible, f"all {visible} CPUs in this process's affinity mask"


def cpu_baseline_legs(args, n):
    """cpu_baseline (1 thread, the reference is serial) and the same path
    batch-parallel over the threads host_threads() names:
    the field says how many threads ran and why, next to the CPUs visible."""
    out = {}
    if args.config == 1 and args.op == "fwd":
        # config 1: the serial single forward of main.cu, for p-I and the
        # reference's own set (BASELINE's q differs from main.cu's)
        out["cpu_baseline"] = cpu_baseline("fwd", args.param, args.cpu_seconds, 1)
        other = "ref" if args.param != "ref" else "p-I"
        out[f"cpu_baseline_{other}"] = cpu_baseline("fwd", other, args.cpu_seconds / 2, 1)
        return out
    out["cpu_baseline"] = cpu_baseline(args.op, args.param, args.cpu_seconds, 1, args.ring)
    threads, visible, why = host_threads()
    par = cpu_baseline(args.op, args.param, args.cpu_seconds / 2, threads, args.ring)
    par["cores_visible"] = visible
    par["threads_reason"] = why
    out["cpu_baseline_parallel"] = par
    if args.op == "nussbaumer":
        # the reference's own Nussbaumer shape: test_nussbaumer, n=1024 mod 2^32-1 (NTT.cu:1987-2005)
        out["cpu_baseline_reference_shape"] = cpu_baseline("nussbaumer", "p-I", args.cpu_seconds / 2, 1, "m32")
    return out


def checker_legs(args, ntt_amd, torch, x, y, z, first, count, n):
    """Correctness legs, outside the timed region.  The oracle (oracle/, the
    CPU restatement of NTT.cu) is only the checker here, as in the tests."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    ps = args.param
    res = {"roundtrip_identity_full_batch": None}
    rng = np.random.default_rng(first + 1)
    # a sampled subset of ~4096 polys plus the first and the last
    # (Nussbaumer's oracle is ~10x slower per product: 1024)
    nsamp = 1024 if args.op == "nussbaumer" else 4096
    idx = np.unique(np.concatenate([[0, count - 1], 1 + rng.choice(count - 2, nsamp - 2, replace=False)])) \
        if count > nsamp else np.arange(count)
    tidx = torch.as_tensor(idx, device=x.device)

    def host(seed, i):   # the device generator's polys, regenerated on the host
        return np.concatenate([O.fill_uniform(1, ps, seed, first + int(k)) for k in i])

    def sample(t):
        return ntt_amd.to_numpy_u32(t.view(count, n)[tidx])

    if args.op == "fwdinv":
        # every step is the identity: the buffer must equal the regenerated input
        ref = torch.empty_like(x)
        ntt_amd.fill_uniform(ref, ps, SEED, first)
        res["roundtrip_identity_full_batch"] = bool(torch.equal(ref, x))
        del ref
    a = host(SEED, idx)
    if args.op in ("fwdinv", "fwd", "inv"):
        # one more launch on the regenerated input, sampled polys vs the oracle
        ntt_amd.fill_uniform(x, ps, SEED, first)
        if args.op == "inv":
            ntt_amd.poly_invntt(x, ps)
            want = O.poly_invntt(a, ps)
        else:
            ntt_amd.poly_ntt(x, ps)
            want = O.poly_ntt(a, ps)
        got = sample(x)
    else:
        b = host(SEED ^ 0xFFFF, idx)
        got = sample(z)
        if args.op == "polymul":
            want = O.poly_mul(a, b, ps)
        elif args.op == "polymul_ntt":   # y is taken as b-hat: c = a * INTT(b-hat)
            want = O.poly_mul(a, O.poly_invntt(b, ps), ps)
        elif args.ring == "m32":
            want = O.m32_canon(O.nussbaumer(a, b, n, "m32"))
        else:
            want = O.poly_mul(a, b, ps)
    res["sampled_vs_oracle"] = {"polys": int(len(idx)), "ok": bool(np.array_equal(got.reshape(want.shape), want))}
    return res


def bench_host(args, ntt_amd, torch, device, rank, world, dist):
    """Host -> host operation through ntt_host_ctx: the
    reference's PCIe-inclusive timing (NTT.cu:2384-2428), pipelined.  Never
    the headline `value` of the device-resident metric."""
    import numpy as np
    pinfo = ntt_amd.param_info(args.param)
    n = pinfo["n"]
    first, count = shard(args.batch, rank)
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
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    dist.barrier()
    elapsed = dist.max(t1 - t0)
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
    dist.close()


if __name__ == "__main__":
    main()
