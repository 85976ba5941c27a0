#!/usr/bin/env python3
"""Per-phase cycle attribution of the Nussbaumer kernel (diagnostic, not the
bench): a library built with -DNUS_STAMPS (tools/build_ab.sh <name> WT
-DNUS_STAMPS ...) records s_memtime at the phase boundaries of each unit
(csrc/nussbaumer.hip, NUS_STAMP) for the first 8192 workgroups; this runs
one p-III mod-q product launch of 2^20 polynomials and prints, per phase,
the mean cycles and share of a unit, separating the pair barriers' waits.

    python tools/nus_stamps.py lib/diag/nus_stamps.so [...]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))

PHASES = [
    "load wait + input scaling", "outer forward (5 stages) + row writes", "barrier 1 (matrices written)",
    "inner level: row reads, inner fwd, 8x8 products, inner inv", "barrier 2 (matrices read)",
    "block results to LDS (+ next unit's loads issued)", "barrier 3 (results written)",
    "recombination reads", "outer inverse (5 stages)", "stage-5 exchange write", "barrier 4 (exchange written)",
    "last stage, output scaling, stores", "barrier 5 (exchange free)",
]


def main():
    import torch
    import ntt_amd
    out = {}
    for path in sys.argv[1:]:
        L = ctypes.CDLL(os.path.abspath(path))
        vp = ctypes.c_void_p
        L.poly_mul_nussbaumer.argtypes = [vp, vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp]
        L.nus_debug_stamps.argtypes = [vp, ctypes.c_size_t]
        batch, n = 1 << 20, 2048
        x = torch.empty(batch * n, dtype=torch.int32, device="cuda")
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        ntt_amd.fill_uniform(x, "p-III", 1)
        ntt_amd.fill_uniform(y, "p-III", 2)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            assert L.poly_mul_nussbaumer(z.data_ptr(), x.data_ptr(), y.data_ptr(), batch, 2, 0, s) == 0
        torch.cuda.synchronize()
        buf = np.zeros((8192 * 2, 16), np.uint64)
        assert L.nus_debug_stamps(buf.ctypes.data, buf.size) == 0
        st = buf[buf[:, 13] > 0].astype(np.float64)
        d = np.diff(st[:, :14], axis=1)
        tot = st[:, 13] - st[:, 0]
        res = {"waves": int(st.shape[0]), "mean_unit_cycles": float(tot.mean()),
               "phases": {PHASES[i]: {"cycles": round(float(d[:, i].mean()), 1),
                                      "share": round(float((d[:, i] / tot).mean()), 4)} for i in range(13)}}
        bar = [2, 4, 6, 10, 12]
        res["barrier_share"] = round(float((d[:, bar].sum(1) / tot).mean()), 4)
        out[os.path.basename(path)] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
