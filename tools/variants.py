#!/usr/bin/env python3
"""Bottleneck attribution for the transform kernels (diagnostic, not the bench).

Times, interleaved in one process (guide rule 24), the production kernel and
its diagnostic variants through ntt_debug_variant of the tools-only library
lib/libqtesla_ntt_diag.so (ntt-gpu-qtesla_amd/tools/ntt_diag.hip, `make tools`):
  full | mem (global load+store only) | alu (no global memory) | lds (load+LDS transpose+store)
plus torch's device copy of the same bytes as an achievable-bandwidth yardstick.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--param", default="p-III")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default=None, help="comma list of names to run")
    args = ap.parse_args()
    import torch
    import ntt_amd
    ntt_amd.lib()   # binds the HIP runtime torch loaded (see ntt_amd.lib)
    L = ctypes.CDLL(os.path.join(ROOT, "ntt-gpu-qtesla_amd", "lib", "libqtesla_ntt_diag.so"))
    L.ntt_debug_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_void_p]
    ps = ntt_amd.PARAM_SETS[args.param]
    n = ntt_amd.param_info(args.param)["n"]
    x = torch.empty(args.batch * n, dtype=torch.int32, device="cuda")
    y = torch.empty_like(x)
    ntt_amd.fill_uniform(x, args.param, 1)
    s = torch.cuda.current_stream()
    names = {}
    for op, opn in ((0, "fwd"), (1, "inv")):
        for v, vn in ((0, "full"), (1, "mem"), (2, "alu"), (3, "lds")):
            names[f"{opn}_{vn}"] = (op, v)
    names["copy_dword"] = (2, 0)
    names["copy_x4"] = (2, 1)
    for v, vn in ((0, "full"), (1, "mem"), (2, "alu")):
        names[f"mul_{vn}"] = (3, v)   # k_poly_mul<PS,false,VAR>: c = x * x
    todo = list(names) + ["torch_copy"]
    if args.only:
        todo = [t for t in todo if t in args.only.split(",")]

    def launch(name):
        if name == "torch_copy":
            y.copy_(x)
            return
        op, v = names[name]
        rc = L.ntt_debug_variant(op, v, y.data_ptr(), x.data_ptr(), args.batch, ps, s.cuda_stream)
        assert rc == 0, rc

    for t in todo:
        launch(t)
    torch.cuda.synchronize()
    res = {t: [] for t in todo}
    for _ in range(args.rounds):
        for t in todo:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch(t)
            e1.record(s)
            e1.synchronize()
            res[t].append(e0.elapsed_time(e1))
    out = {}
    for t, v in res.items():
        v.sort()
        med = v[len(v) // 2]
        bytes_ = args.batch * n * (12 if t.startswith("mul_") else 8)
        out[t] = {"ms_median": med, "ms_min": v[0], "GBps_alg": bytes_ / (med * 1e-3) / 1e9}
    bytes_ = args.batch * n * 8
    print(json.dumps({"param": args.param, "batch": args.batch, "bytes_per_launch": bytes_, "results": out}, indent=1))


if __name__ == "__main__":
    main()
