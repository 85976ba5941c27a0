#!/usr/bin/env python3
"""Summarise two rocprofv3 PMC passes of one bench.py configuration into
profiles/pmc_summary.json (one entry per workload, stamped with the library
build hash so that bench.py reports `traffic` only for the build measured).

    python tools/pmc_summary.py --fetch F.csv --write W.csv --config 3 [--op ... --param ... --batch ...]

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KiB;
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads exactly half the bytes
of a coalesced streaming read, so it is doubled; WRITE_SIZE is exact).
Median over the profiled launches of each kernel; the dominant (largest)
kernel's bytes are the entry's hbm_bytes_per_launch.
"""
import argparse
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def load(path):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        out[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return out


def kernel_patterns(op, ps, ring, radix=None):
    """rocprof kernel-name patterns of a bench op's launches.  radix: the
    small-batch family the transforms run at this batch (ntt_small_batch_radix:
    4 / 8 / 16 = the one-polynomial-per-workgroup kernels, 0 / None = the
    batch kernels)."""
    if op in ("fwdinv", "fwd", "inv") and radix:
        kern = (lambda inv: f"k_ntt_lat<{ps}, {inv}, false>") if radix == 4 else \
            (lambda inv: f"k_ntt_latr<{ps}, {inv}, false, {3 if radix == 8 else 4}, 0>")
        return {"fwdinv": {"fwd": kern("false"), "inv": kern("true")}, "fwd": {"fwd": kern("false")},
                "inv": {"inv": kern("true")}}[op]
    if ps >= 3:   # n = 4096 / 8192: wave-per-polynomial transforms (and n = 4096 products),
        # the n = 8192 products on the multi-wave four-step kernel
        mk = "k_poly_mul_big" if ps == 3 else "k_poly_mul_large"
        return {"fwdinv": {"fwd": f"k_ntt_fwd_big<{ps}, false>", "inv": f"k_ntt_inv_big<{ps}, false>"},
                "fwd": {"fwd": f"k_ntt_fwd_big<{ps}, false>"}, "inv": {"inv": f"k_ntt_inv_big<{ps}, false>"},
                "polymul": {"mul": f"{mk}<{ps}, false>"},
                "polymul_ntt": {"mulntt": f"{mk}<{ps}, true>"}}[op]
    return {"fwdinv": {"fwd": f"k_ntt_fwd<{ps}, false>", "inv": f"k_ntt_inv<{ps}, false>"},
            "fwd": {"fwd": f"k_ntt_fwd<{ps}, false>"}, "inv": {"inv": f"k_ntt_inv<{ps}, false>"},
            "polymul": {"mul": f"k_poly_mul<{ps}, false, 0>"}, "polymul_ntt": {"mulntt": f"k_poly_mul<{ps}, true, 0>"},
            "nussbaumer": {"nus": f"k_nussbaumer<{ps if not (ring == 'm32' and ps == 0) else 1}, "
                                  f"{1 if ring == 'm32' else 0}>"}}[op]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--op")
    ap.add_argument("--param")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--ring")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
    args = ap.parse_args()
    import bench
    import ntt_amd
    c_op, c_param, c_batch, c_ring = bench.CONFIGS[args.config]
    op, param, batch, ring = args.op or c_op, args.param or c_param, args.batch or c_batch, args.ring or c_ring
    info = ntt_amd.param_info(param)
    n = info["n"]
    ps = ntt_amd.PARAM_SETS[param]
    workload = bench.workload_name(op, param, n, info["q"], ring)
    alg = batch * n * (12 if op in ("polymul", "polymul_ntt", "nussbaumer") else 8)
    f, w = load(args.fetch), load(args.write)
    kernels = {}
    radix = None
    if op in ("fwdinv", "fwd", "inv"):
        radices = {ntt_amd.small_batch_radix(param, k, batch) for k in bench.SWITCH_OPS[op]}
        radix = radices.pop() if len(radices) == 1 else None
    for key, pat in kernel_patterns(op, ps, ring, radix).items():
        fk = [v for (k, c), v in f.items() if c == "FETCH_SIZE" and pat in k]
        wk = [v for (k, c), v in w.items() if c == "WRITE_SIZE" and pat in k]
        if not fk or not wk:
            continue
        fetch_kib, write_kib = statistics.median(fk[0]), statistics.median(wk[0])
        hbm = (2 * fetch_kib + write_kib) * 1024
        kernels[key] = {"kernel": pat, "launches": len(fk[0]), "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
                        "hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / alg}
    if not kernels:
        sys.exit(f"no {op} kernel found in {args.fetch} / {args.write}")
    entry = {"workload": workload, "op": op, "param": param, "batch": batch, "n": n, "alg_bytes_per_launch": alg,
             "build_hash": ntt_amd.build_hash(), "kernels": kernels,
             "hbm_bytes_per_launch": max(v["hbm_bytes_per_launch"] for v in kernels.values()),
             "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of the same bench command; "
                       "2 x FETCH_SIZE + WRITE_SIZE (KiB), median over launches"}
    try:
        d = json.load(open(args.out))
    except (OSError, ValueError):
        d = {}
    d.setdefault("entries", {})[workload] = entry
    json.dump(d, open(args.out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
