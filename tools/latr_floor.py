#!/usr/bin/env python3
"""Memory-only floors of the two n <= 2048 transform geometries at a batch
(diagnostic, not the bench), interleaved in one process on the same buffers
(tools/ntt_diag.hip, `make tools`):
  batch kernels (wave per polynomial, 8 KiB stored per wave): ntt_debug_variant
      op 0 / 1 (fwd / inv), variant 0 = full, 3 = loads + LDS transpose + stores
  radix-8 / radix-16 workgroup per polynomial (csrc/ntt_latr.hpp, 2 / 4 KiB
      per wave): op 5 / 6, variants 0-3 forward, 4-7 inverse: full, memory
      only (loads + LDS exchanges and barriers + stores), arithmetic + twiddle
      loads + LDS only, memory only plus the twiddle loads
Each point: an event pair around `steps` back-to-back launches, median over rounds.

    python tools/latr_floor.py [--param p-III] [--batch 1048576] [--steps 10] [--rounds 7]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--param", default="p-III")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--oop", action="store_true", help="write to a second buffer (default: in place, as bench.py)")
    args = ap.parse_args()
    import torch
    import ntt_amd
    D = ctypes.CDLL(os.path.join(ROOT, "ntt-gpu-qtesla_amd", "lib", "libqtesla_ntt_diag.so"))
    vp = ctypes.c_void_p
    D.ntt_debug_variant.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    ps = ntt_amd.PARAM_SETS[args.param]
    n = ntt_amd.param_info(args.param)["n"]
    x = torch.empty(args.batch * n, dtype=torch.int32, device="cuda")
    ntt_amd.fill_uniform(x, args.param, 5)
    y = torch.empty_like(x) if args.oop else x
    s = torch.cuda.current_stream()
    cases = {"batch_fwd_full": (0, 0), "batch_fwd_mem": (0, 3), "batch_inv_full": (1, 0), "batch_inv_mem": (1, 3)}
    for op, nm in ((5, "r8"), (6, "r16")):
        for d, base in (("fwd", 0), ("inv", 4)):
            for v, kind in enumerate(("full", "mem", "alu", "memtw")):
                cases[f"{nm}_{d}_{kind}"] = (op, base + v)

    def run(op, var):
        rc = D.ntt_debug_variant(op, var, vp(y.data_ptr()), vp(x.data_ptr()), args.batch, ps, vp(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"variant {op}/{var}: {rc}")
    for c in cases.values():
        run(*c)
    torch.cuda.synchronize()
    t = {k: [] for k in cases}
    for _ in range(args.rounds):
        for k, c in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.steps):
                run(*c)
            e1.record(s)
            e1.synchronize()
            t[k].append(e0.elapsed_time(e1) / args.steps)
    alg = 8 * n * args.batch
    out = {k: {"ms": round(statistics.median(v), 4), "frac_of_8TBs": round(alg / (statistics.median(v) * 1e-3) / 8e12, 4)}
           for k, v in t.items()}
    print(json.dumps({"param": args.param, "batch": args.batch, "steps": args.steps, "rounds": args.rounds,
                      "inplace": not args.oop,
                      "results": out}, indent=1))


if __name__ == "__main__":
    main()
