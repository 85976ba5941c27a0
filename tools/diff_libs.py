#!/usr/bin/env python3
"""Diagnostic: run poly_ntt_oop / poly_invntt_oop of two library builds on the
same device input several times and report which polynomials / 2048-word
blocks differ (determinism and location of a mismatch).

    python tools/diff_libs.py A.so B.so --param p-III-8192 --batch 262144 [--reps 3]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--param", default="p-III-8192")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--inplace", action="store_true", help="out == in (a copy of the input per run)")
    args = ap.parse_args()
    import torch
    import ntt_amd
    ps = ntt_amd.PARAM_SETS[args.param]
    n = ntt_amd.param_info(args.param)["n"]
    libs = [ctypes.CDLL(os.path.abspath(p)) for p in (args.a, args.b)]
    for L in libs:
        for nm in ("poly_ntt_oop", "poly_invntt_oop"):
            getattr(L, nm).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    x = torch.empty(args.batch * n, dtype=torch.int32, device=dev)
    ntt_amd.fill_uniform(x, args.param, 0x5EED0042, 0)
    for op in ("poly_ntt_oop", "poly_invntt_oop"):
        outs = []
        for L in libs:
            for r in range(args.reps):
                y = x.clone() if args.inplace else torch.empty_like(x)
                src = y if args.inplace else x
                assert getattr(L, op)(y.data_ptr(), src.data_ptr(), args.batch, ps, None) == 0
                torch.cuda.synchronize()
                outs.append(y.view(args.batch, n))
        ref = outs[0]
        for i, o in enumerate(outs):
            bad = (o != ref).any(dim=1).nonzero().flatten()
            blocks = sorted(set(((o != ref).view(args.batch, n // 2048, 2048).any(dim=2).nonzero()[:, 1]).tolist()))
            print(op, "lib", i // args.reps, "rep", i % args.reps, "bad polys", bad.numel(),
                  bad[:8].tolist(), "blocks", blocks, flush=True)


if __name__ == "__main__":
    main()
