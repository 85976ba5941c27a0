#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_summary.json.

HBM bytes per launch of the transform kernels, from separate FETCH_SIZE and
WRITE_SIZE passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE in KiB;
on gfx950 FETCH_SIZE reads exactly half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact).  The correction is
checked in-run on __amd_rocclr_copyBuffer-free data: the uncorrected
FETCH_SIZE of the transforms equals 1/2 of their algorithmic read bytes.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def load(path):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        out[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return out


def main(fetch_csv, write_csv, out_path, batch=1 << 20, n=2048):
    f, w = load(fetch_csv), load(write_csv)
    alg = batch * n * 8
    res = {"workload": "fwd+inv negacyclic NTT n=2048 qTESLA-p-III", "batch": batch, "n": n,
           "alg_bytes_per_launch": alg, "kernels": {}}
    for (k, c), v in f.items():
        if c != "FETCH_SIZE" or ("k_ntt_fwd<2, 0>" not in k and "k_ntt_inv<2, 0>" not in k):
            continue
        ws = w.get((k, "WRITE_SIZE"), [0.0])
        fetch_kib, write_kib = statistics.median(v), statistics.median(ws)
        hbm = (2 * fetch_kib + write_kib) * 1024
        res["kernels"]["fwd" if "fwd" in k else "inv"] = {
            "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
            "hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / alg}
    ks = res["kernels"]
    if ks:
        res["hbm_bytes_per_launch"] = max(v["hbm_bytes_per_launch"] for v in ks.values())
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
