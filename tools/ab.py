#!/usr/bin/env python3
"""Interleaved A/B of library builds in ONE process (diagnostic, not the bench).

Loads every .so given (e.g. ntt-gpu-qtesla_amd/lib/ab/*.so, built with
different -D switches) side by side through ctypes and times poly_ntt /
poly_invntt / poly_mul of each on the same device buffers, round-robin, so
that clock / thermal drift hits all builds alike (guide rule 24).  Each
build's output is checked against the first build's.

    python tools/ab.py lib1.so lib2.so ... [--ops fwd,inv] [--rounds 7]
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--param", default="p-III")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--ops", default="fwd,inv")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--inplace", action="store_true", help="transform x in place (as bench.py does)")
    args = ap.parse_args()
    import torch
    import ntt_amd
    ps = ntt_amd.PARAM_SETS[args.param]
    n = ntt_amd.param_info(args.param)["n"]
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    libs = {}
    for path in args.libs:
        L = ctypes.CDLL(os.path.abspath(path))
        for nm in ("poly_ntt_oop", "poly_invntt_oop", "poly_bitrev_copy", "poly_ntt_bitrev", "poly_invntt_bitrev"):
            getattr(L, nm).argtypes = [vp, vp, sz, ctypes.c_int, vp]
        L.poly_mul.argtypes = [vp, vp, vp, sz, ctypes.c_int, vp]
        L.poly_mul_ntt.argtypes = [vp, vp, vp, sz, ctypes.c_int, vp]
        L.poly_mul_nussbaumer.argtypes = [vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
        libs[os.path.basename(path)] = L
    x = torch.empty(args.batch * n, dtype=torch.int32, device="cuda")
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    ntt_amd.fill_uniform(x, args.param, 11)
    ntt_amd.fill_uniform(y, args.param, 12)
    s = torch.cuda.current_stream()
    ops = args.ops.split(",")

    def launch(L, op):
        dst = x if args.inplace else z
        if op == "fwd":
            rc = L.poly_ntt_oop(dst.data_ptr(), x.data_ptr(), args.batch, ps, s.cuda_stream)
        elif op == "inv":
            rc = L.poly_invntt_oop(dst.data_ptr(), x.data_ptr(), args.batch, ps, s.cuda_stream)
        elif op in ("bitrev", "fwdbr", "invbr"):
            fn = {"bitrev": L.poly_bitrev_copy, "fwdbr": L.poly_ntt_bitrev, "invbr": L.poly_invntt_bitrev}[op]
            rc = fn(dst.data_ptr(), x.data_ptr(), args.batch, ps, s.cuda_stream)
        elif op in ("nus", "nusm32"):
            rc = L.poly_mul_nussbaumer(z.data_ptr(), x.data_ptr(), y.data_ptr(), args.batch, ps, 1 if op == "nusm32" else 0,
                                       s.cuda_stream)
        elif op == "mulntt":
            rc = L.poly_mul_ntt(z.data_ptr(), x.data_ptr(), y.data_ptr(), args.batch, ps, s.cuda_stream)
        else:
            rc = L.poly_mul(z.data_ptr(), x.data_ptr(), y.data_ptr(), args.batch, ps, s.cuda_stream)
        assert rc == 0, rc

    ref = {}
    ok = {}
    for name, L in libs.items():
        for op in ops:
            launch(L, op)
            torch.cuda.synchronize()
            sig = (x if args.inplace and op in ("fwd", "inv", "bitrev", "fwdbr", "invbr") else z)[:: 4099].clone()
            if op not in ref:
                ref[op] = sig
            ok[f"{name}:{op}"] = bool(torch.equal(ref[op], sig))
    times = {f"{name}:{op}": [] for name in libs for op in ops}
    for _ in range(args.rounds):
        for name, L in libs.items():
            for op in ops:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                launch(L, op)
                e1.record(s)
                e1.synchronize()
                times[f"{name}:{op}"].append(e0.elapsed_time(e1))
    out = {k: {"ms_median": statistics.median(v), "ms_min": min(v), "matches_first": ok[k]} for k, v in times.items()}
    print(json.dumps({"param": args.param, "batch": args.batch, "inplace": args.inplace, "results": out}, indent=1))


if __name__ == "__main__":
    main()
