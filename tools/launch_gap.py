#!/usr/bin/env python3
"""Back-to-back launch overhead of one in-place transform (diagnostic, not the
bench): K launches of poly_ntt on the same buffer timed by one event pair
(plain stream launches), and the same K launches captured once into a HIP
graph and replayed.  With --trace CSV (a rocprofv3 --kernel-trace of this
script), prints the kernels' own durations and the idle gaps between them.

    python tools/launch_gap.py [--param p-I --batch 65536 --k 40]
    python tools/launch_gap.py --trace gpurun_out/gap/run_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def trace(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_ntt_fwd" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    small = [g for g in gap if g < 50]   # back-to-back launches only (not the host-side pauses between phases)
    print(json.dumps({"kernels": len(rows), "dur_us_median": statistics.median(dur), "dur_us_min": min(dur),
                      "gap_us_median_back_to_back": statistics.median(small) if small else None,
                      "gap_us_min": min(small) if small else None, "gaps_counted": len(small)}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--param", default="p-I")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--trace")
    ap.add_argument("--default-stream", action="store_true", help="launch on the null stream (bench.py's r03 setup)")
    args = ap.parse_args()
    if args.trace:
        return trace(args.trace)
    import torch
    import ntt_amd
    n = ntt_amd.param_info(args.param)["n"]
    x = torch.empty(args.batch * n, dtype=torch.int32, device="cuda")
    ntt_amd.fill_uniform(x, args.param, 7)
    s = torch.cuda.default_stream() if args.default_stream else torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(5):
            ntt_amd.poly_ntt(x, args.param, s)
    torch.cuda.synchronize()
    g = None
    if not args.default_stream:   # (capture needs a side stream)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(args.k):
                ntt_amd.poly_ntt(x, args.param, s)
        torch.cuda.synchronize()

    def region(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            fn()
            e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.k * 1e3   # us per launch

    def plain():
        for _ in range(args.k):
            ntt_amd.poly_ntt(x, args.param, s)

    res = {"plain_us": [], "graph_us": []}
    for _ in range(args.rounds):
        res["plain_us"].append(region(plain))
        if g is not None:
            res["graph_us"].append(region(g.replay))
    out = {"param": args.param, "batch": args.batch, "k": args.k}
    out["stream"] = "null" if args.default_stream else "created"
    for kname, v in res.items():
        if v:
            out[kname] = {"median": statistics.median(v), "min": min(v)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
