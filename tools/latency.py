#!/usr/bin/env python3
"""Small-batch latency of the transforms (diagnostic, not the bench): the
qTESLA signing loop transforms ONE polynomial per call, so BASELINE config 1
(batch 1) is a latency measurement, not a bandwidth one.

For each case and batch, interleaved over rounds in one process:
  gpu_us  = one HIP event pair around `steps` back-to-back launches on one
            stream, / steps (what bench.py's config-1 line reports as the
            launch time),
  wall_us = host wall time of the same loop / steps (the Python -> C-ABI ->
            hipLaunchKernel cost when it exceeds the GPU time).
  graph_us = the same `steps` launches captured once in a HIP graph (torch.cuda.CUDAGraph)
            and replayed: the GPU time per launch without the host's
            submission cost (a C caller's steady state, kernel + boundary).
Cases: the product entry points (poly_ntt / poly_invntt / poly_mul), the
diagnostic library's memory-only variant of the same forward kernel
(ntt_debug_variant op 0 variant 1) and its workgroup-per-polynomial n = 2048
forward (op 4 variant 1), and a one-element torch add (the launch floor).

    python tools/latency.py [--batches 1,8,64] [--steps 200] [--rounds 5] [--lib L.so ...]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,64")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default=None, help="product library to load instead of the in-tree one")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--params", default="p-I,p-III")
    args = ap.parse_args()
    if args.lib:
        os.environ["NTT_AMD_LIB"] = args.lib
    import torch
    import ntt_amd
    ntt_amd.lib()
    cur = lambda: torch.cuda.current_stream()   # noqa: E731 (graph capture runs on its own stream)
    D = ctypes.CDLL(os.path.join(ROOT, "ntt-gpu-qtesla_amd", "lib", "libqtesla_ntt_diag.so"))
    D.ntt_debug_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_void_p]
    s = torch.cuda.current_stream()
    batches = [int(b) for b in args.batches.split(",")]
    bufs = {}
    params = args.params.split(",")
    for param in params:
        n = ntt_amd.param_info(param)["n"]
        for b in batches:
            x = torch.empty(b * n, dtype=torch.int32, device="cuda")
            ntt_amd.fill_uniform(x, param, 7)
            bufs[param, b] = (x, torch.empty_like(x), torch.empty_like(x))
    one = torch.zeros(1, dtype=torch.int32, device="cuda")

    def case(name, param, b):
        if name == "torch_add_1":
            return lambda: one.add_(1)
        x, y, z = bufs[param, b]
        ps = ntt_amd.PARAM_SETS[param]
        if name == "poly_ntt":
            return lambda: ntt_amd.poly_ntt(x, param, cur())
        if name == "poly_invntt":
            return lambda: ntt_amd.poly_invntt(x, param, cur())
        if name == "poly_mul":
            return lambda: ntt_amd.poly_mul(z, x, y, param, cur())
        if name == "poly_ntt_ctypes":   # the C ABI straight from ctypes: the wrapper's own cost is the difference
            L, ptr, psn = ntt_amd.lib(), x.data_ptr(), ntt_amd.PARAM_SETS[param]
            return lambda: L.poly_ntt(ptr, None, b, psn, cur().cuda_stream)
        if name == "fwd_mem_only":
            return lambda: D.ntt_debug_variant(0, 1, y.data_ptr(), x.data_ptr(), b, ps, cur().cuda_stream)
        if name == "fwd_wg_per_poly":
            return lambda: D.ntt_debug_variant(4, 1, y.data_ptr(), x.data_ptr(), b, ps, cur().cuda_stream)
        raise KeyError(name)

    todo = []
    for b in batches:
        for param in params:
            for name in ("poly_ntt", "poly_ntt_ctypes", "poly_invntt", "poly_mul", "fwd_mem_only"):
                if name == "fwd_mem_only" and ntt_amd.param_info(param)["n"] > 2048:
                    continue   # the diagnostic variants are n <= 2048
                todo.append((name, param, b))
            if param == "p-III":
                todo.append(("fwd_wg_per_poly", param, b))
    todo.append(("torch_add_1", "-", 1))
    fns = {t: case(*t) for t in todo}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    graphs = {}
    if not args.no_graph:
        for t in todo:
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(args.steps):
                        fns[t]()
                graphs[t] = g
            except Exception as e:   # noqa: BLE001 (reported, the other legs still run)
                graphs[t] = f"{type(e).__name__}: {e}"
        torch.cuda.synchronize()
    res = {t: {"gpu": [], "wall": [], "graph": []} for t in todo}
    for _ in range(args.rounds):
        for t in todo:
            f = fns[t]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            e0.record(s)
            for _ in range(args.steps):
                f()
            e1.record(s)
            w1 = time.perf_counter()
            torch.cuda.synchronize()
            res[t]["gpu"].append(e0.elapsed_time(e1) * 1e3 / args.steps)
            res[t]["wall"].append((w1 - w0) * 1e6 / args.steps)
            g = graphs.get(t)
            if g is not None and not isinstance(g, str):
                g.replay()   # warm
                e0.record(s)
                g.replay()
                e1.record(s)
                torch.cuda.synchronize()
                res[t]["graph"].append(e0.elapsed_time(e1) * 1e3 / args.steps)
    out = {}
    for t, r in res.items():
        o = out[f"{t[0]}:{t[1]}:b{t[2]}"] = {"gpu_us": round(statistics.median(r["gpu"]), 3),
                                             "wall_us": round(statistics.median(r["wall"]), 3)}
        if r["graph"]:
            o["graph_us"] = round(statistics.median(r["graph"]), 3)
        elif isinstance(graphs.get(t), str):
            o["graph_error"] = graphs[t]
    print(json.dumps({"steps": args.steps, "rounds": args.rounds, "lib": ntt_amd.build_info(), "cases": out},
                     indent=1))


if __name__ == "__main__":
    main()
