"""Per-call cost of the Python entry points at batch 1 (config 1's shape):
the ntt_amd wrapper against a bare ctypes call of the same C-ABI function,
on one stream, synchronised once per 2000 calls.  Prints JSON."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))
import torch  # noqa: E402
import ntt_amd  # noqa: E402


def rate(fn, calls=2000, rounds=5):
    best = None
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / calls * 1e6
        best = dt if best is None else min(best, dt)
    return best


def main():
    x = torch.zeros(1024, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    L = ntt_amd.lib()
    ps = ntt_amd.PARAM_SETS["p-I"]
    ptr, sp = x.data_ptr(), st.cuda_stream
    out = {
        "wrapper_us": rate(lambda: ntt_amd.poly_ntt(x, "p-I", st)),
        "wrapper_default_stream_us": rate(lambda: ntt_amd.poly_ntt(x, "p-I")),
        "bare_ctypes_us": rate(lambda: L.poly_ntt(ptr, None, 1, ps, sp)),
        "python_loop_us": rate(lambda: None),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
