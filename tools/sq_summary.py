#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counter summary of rocprofv3 --pmc runs (medians over
launches).  Derived: VALU issue share = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES
per SIMD, and effective clock = GRBM_GUI_ACTIVE / 8 / kernel time when a
kernel-trace duration is supplied (MI355X_MICROARCH.md, DVFS).

    python tools/sq_summary.py run_counter_collection.csv [more.csv ...]
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        if "fill_uniform" in k or "rocclr" in k:
            continue
        out[k] = {c: statistics.median(v) for c, v in sorted(cs.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
