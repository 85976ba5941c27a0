#!/usr/bin/env python3
"""Small-batch switch sweep (diagnostic, not the bench): times the latency
kernels (one polynomial per workgroup, csrc/ntt_lat.hpp) against the batch
kernels at doubling batches, for every parameter set and switching entry
point, so that the switch (csrc/ntt_lat.hpp lat_max_polys) is set per
(n, op) from the measured crossover.

The two paths come from two A/B builds of the same sources
(tools/build_ab.sh): one with every batch on the batch kernels
(-DNTT_LAT_FORCE=0), one with every batch on the latency kernels
(-DNTT_LAT_FORCE=1).  Both are loaded side by side in ONE process and
timed round-robin on the same buffers (clock drift hits both alike); each
point is one HIP event pair around K back-to-back launches (K sized so the
region is >= ~2 ms, at most 200), median over rounds.  Outputs are checked
equal between the builds.

    python tools/switch_sweep.py BATCH.so SMALL.so [SMALL2.so ...] [--params p-I,p-III] [--ops fwd,inv,...]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))

# largest batch per n: the BASELINE batches (config 3: 2^20 at n = 2048) and
# 8 GiB per array at n = 4096 / 8192
MAX_BATCH = {1024: 1 << 20, 2048: 1 << 20, 4096: 1 << 19, 8192: 1 << 18}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch_lib")
    ap.add_argument("lat_lib", nargs="+", help="one or more builds whose small-batch path to compare (tag = file name)")
    ap.add_argument("--params", default="p-I,p-III,p-III-4096,p-III-8192")
    ap.add_argument("--ops", default="fwd,inv,fwdbr,invbr,mul,mulntt")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-batch", type=int, default=64)
    ap.add_argument("--max-batch", type=int, default=0, help="cap (0: MAX_BATCH per n)")
    ap.add_argument("--target-ms", type=float, default=2.0)
    ap.add_argument("--inplace", action="store_true",
                    help="fwd / inv in place (poly_ntt / poly_invntt, as bench.py runs them); default out of place")
    ap.add_argument("--out", default=None)
    ap.add_argument("--refine", default=None,
                    help="a previous sweep's JSON: time 8 points per octave inside each (n, op)'s crossover octave")
    args = ap.parse_args()
    import torch
    import ntt_amd
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    libs = {}
    for tag, path in [("batch", args.batch_lib)] + [(os.path.basename(p)[:-3], p) for p in args.lat_lib]:
        L = ctypes.CDLL(os.path.abspath(path))
        for nm in ("poly_ntt_oop", "poly_invntt_oop", "poly_ntt_bitrev", "poly_invntt_bitrev"):
            getattr(L, nm).argtypes = [vp, vp, sz, ctypes.c_int, vp]
        for nm in ("poly_mul", "poly_mul_ntt"):
            getattr(L, nm).argtypes = [vp, vp, vp, sz, ctypes.c_int, vp]
        libs[tag] = L
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    res = {}
    t_start = time.time()
    for param in args.params.split(","):
        ps = ntt_amd.PARAM_SETS[param]
        n = ntt_amd.param_info(param)["n"]
        top = MAX_BATCH[n] if not args.max_batch else min(args.max_batch, MAX_BATCH[n])
        x = torch.empty(top * n, dtype=torch.int32, device="cuda")
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        ntt_amd.fill_uniform(x, param, 21)
        ntt_amd.fill_uniform(y, param, 22)
        for op in args.ops.split(","):
            if op in ("mul", "mulntt") and n > 4096:
                continue   # no latency product at n = 8192
            if args.refine:
                prev = json.load(open(args.refine))["summary"]
                # a set the coarse sweep skipped (ref) takes the octave of its n's other set (p-I)
                key = f"{param}:{op}" if f"{param}:{op}" in prev else f"p-I:{op}"
                lo = prev.get(key, {}).get("lat_wins_through", 0)
                if lo == 0 or lo >= top:
                    continue
                batches = [lo + k * lo // 8 for k in range(9)]
            else:
                batches = []
                b = args.min_batch
                while b <= top:
                    batches.append(b)
                    b *= 2
            for b in batches:
                def launch(L, op=op, b=b):
                    dst = x if args.inplace else z
                    if op == "fwd":
                        rc = L.poly_ntt_oop(dst.data_ptr(), x.data_ptr(), b, ps, sp)
                    elif op == "inv":
                        rc = L.poly_invntt_oop(dst.data_ptr(), x.data_ptr(), b, ps, sp)
                    elif op == "fwdbr":
                        rc = L.poly_ntt_bitrev(z.data_ptr(), x.data_ptr(), b, ps, sp)
                    elif op == "invbr":
                        rc = L.poly_invntt_bitrev(z.data_ptr(), x.data_ptr(), b, ps, sp)
                    elif op == "mul":
                        rc = L.poly_mul(z.data_ptr(), x.data_ptr(), y.data_ptr(), b, ps, sp)
                    else:
                        rc = L.poly_mul_ntt(z.data_ptr(), x.data_ptr(), y.data_ptr(), b, ps, sp)
                    if rc != 0:
                        raise RuntimeError(f"{op} b={b} rc={rc}")
                sig = {}
                if args.inplace and op in ("fwd", "inv"):
                    x0 = x[: b * n].clone()
                for tag, L in libs.items():
                    if args.inplace and op in ("fwd", "inv"):
                        x[: b * n].copy_(x0)
                    launch(L)
                    torch.cuda.synchronize()
                    sig[tag] = (x if args.inplace and op in ("fwd", "inv") else z)[: b * n: 4099].clone()
                same = all(bool(torch.equal(sig["batch"], v)) for v in sig.values())
                if args.inplace and op in ("fwd", "inv"):
                    del x0
                # one probe launch of the batch build sizes K
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                launch(libs["batch"])
                e1.record(s)
                e1.synchronize()
                one = max(e0.elapsed_time(e1), 1e-3)
                k = int(max(3, min(200, args.target_ms / one)))
                times = {tag: [] for tag in libs}
                for _ in range(args.rounds):
                    for tag, L in libs.items():
                        e0.record(s)
                        for _ in range(k):
                            launch(L)
                        e1.record(s)
                        e1.synchronize()
                        times[tag].append(e0.elapsed_time(e1) * 1e3 / k)
                r = {tag: round(statistics.median(v), 3) for tag, v in times.items()}
                r["k"] = k
                r["same"] = same
                res.setdefault(param, {}).setdefault(op, {})[b] = r
                print(f"[{time.time() - t_start:6.1f}s] {param} {op} b={b}: " +
                      ", ".join(f"{tag} {r[tag]} us" for tag in libs) + f", same={same}", flush=True)
        del x, y, z
        torch.cuda.empty_cache()
    # per (n, op): the fastest build at every batch, and for each small-batch
    # build the largest batch up to which it beats the batch kernels at every
    # measured point (the switch is one threshold per (n, op))
    summary = {}
    for param, ops in res.items():
        for op, pts in ops.items():
            ent = {"fastest": {str(b): min((t for t in libs), key=lambda t: pts[b][t]) for b in sorted(pts)}}
            for tag in libs:
                if tag == "batch":
                    continue
                last_win = 0
                for b in sorted(pts):
                    if pts[b][tag] < pts[b]["batch"]:
                        last_win = b
                    else:
                        break
                ent[tag] = {"wins_through": last_win,
                            "wins_at": [b for b in sorted(pts) if pts[b][tag] < pts[b]["batch"]]}
            # round 5/6 field name for the radix-4 build (b_lat)
            first = next(t for t in libs if t != "batch")
            ent["lat_wins_through"] = ent[first]["wins_through"]
            summary[f"{param}:{op}"] = ent
    out = {"rounds": args.rounds, "inplace": args.inplace, "libs": {"batch": args.batch_lib, "small": args.lat_lib},
           "results": {p: {o: {str(b): v for b, v in pts.items()} for o, pts in ops.items()} for p, ops in res.items()},
           "summary": summary}
    txt = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
