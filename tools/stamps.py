#!/usr/bin/env python3
"""Per-phase cycle shares of the forward kernel (diagnostic stamped variants,
in-kernel s_memtime; guide §7 'In-kernel stamps').  Read shares, not lengths."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))


def main():
    import torch
    import ntt_amd
    L = ntt_amd.lib()
    L.ntt_debug_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_void_p]
    ps, batch = 2, 1 << 20
    n = 2048
    x = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    ntt_amd.fill_uniform(x, "p-III", 3)
    out = {}
    for v, name in ((4, "full"), (5, "alu")):
        y = torch.zeros(batch * n, dtype=torch.int32, device="cuda")
        for _ in range(2):
            assert L.ntt_debug_variant(0, v, y.data_ptr(), x.data_ptr(), batch, ps,
                                       torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        st = y[: 4096 * 16].cpu().numpy().view(np.uint64).reshape(-1, 8)
        st = st[st[:, 4] > 0]
        tot = st[:, 4].astype(np.float64)
        ph = st[:, :4].astype(np.float64)
        names = ["pass1+swap(+load wait)", "lds_transpose", "pass2", "reduce+store"]
        out[name] = {"waves": int(st.shape[0]), "mean_total_cycles": float(tot.mean()),
                     "shares": {names[i]: float((ph[:, i] / tot).mean()) for i in range(4)},
                     "loop_overhead_share": float(1 - (ph.sum(1) / tot).mean())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
