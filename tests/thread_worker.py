"""Fresh-process worker of tests/test_gpu_threads.py: NTHREADS host threads
make their FIRST library calls at the same moment (a threading.Barrier
releases them together; ctypes drops the GIL for the call), each on its own
HIP stream of the same device and its own buffers, then keep launching
poly_ntt / poly_invntt / poly_mul for several rounds.  Prints one JSON line
with each thread's bit-exact verdicts against the oracle.

Reference: the reference drives everything from one host thread on the
default stream (NTT.cu:2385-2426); the ABI promises reentrancy across
streams and devices (include/qtesla_ntt.h)."""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ntt-gpu-qtesla_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ntt_amd  # noqa: E402
import oracle as O  # noqa: E402

NTHREADS = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ROUNDS = 6
SETS = ["p-III", "p-I", "ref", "p-III-4096", "p-III-8192"]


def main():
    dev = torch.device("cuda:0")
    L = ntt_amd.lib()
    jobs = []
    for t in range(NTHREADS):
        ps = SETS[t % len(SETS)]
        batch = 37 + 64 * t
        a = O.fill_uniform(batch, ps, 0x7000 + t, 0)
        b = O.fill_uniform(batch, ps, 0x7100 + t, 0)
        jobs.append(dict(ps=ps, psi=ntt_amd.PARAM_SETS[ps], batch=batch, a=a, b=b,
                         stream=torch.cuda.Stream(dev),
                         ta=ntt_amd.from_numpy_u32(a, dev), tb=ntt_amd.from_numpy_u32(b, dev),
                         x=ntt_amd.from_numpy_u32(a, dev), c=torch.empty(a.size, dtype=torch.int32, device=dev),
                         rcs=[]))
    torch.cuda.synchronize()
    gate = threading.Barrier(NTHREADS)

    def run(j):
        s = j["stream"].cuda_stream
        gate.wait()
        for r in range(ROUNDS):
            # the first call of every thread is its first library call at all
            j["rcs"].append(L.poly_ntt(j["x"].data_ptr(), None, j["batch"], j["psi"], s))
            if r == ROUNDS - 1:
                break        # leave x in the NTT domain after the last round
            j["rcs"].append(L.poly_invntt(j["x"].data_ptr(), None, j["batch"], j["psi"], s))
            j["rcs"].append(L.poly_mul(j["c"].data_ptr(), j["ta"].data_ptr(), j["tb"].data_ptr(), j["batch"],
                                       j["psi"], s))

    threads = [threading.Thread(target=run, args=(j,)) for j in jobs]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    torch.cuda.synchronize()
    out = []
    for j in jobs:
        ok_rc = all(rc == 0 for rc in j["rcs"])
        ok_ntt = bool(np.array_equal(ntt_amd.to_numpy_u32(j["x"]).reshape(j["a"].shape), O.poly_ntt(j["a"], j["ps"])))
        ok_mul = bool(np.array_equal(ntt_amd.to_numpy_u32(j["c"]).reshape(j["a"].shape),
                                     O.poly_mul(j["a"], j["b"], j["ps"])))
        out.append(dict(ps=j["ps"], batch=j["batch"], rc_ok=ok_rc, ntt=ok_ntt, mul=ok_mul, calls=len(j["rcs"])))
    print(json.dumps({"threads": out, "expiries": ntt_amd.sync_expiries()}), flush=True)


if __name__ == "__main__":
    main()
