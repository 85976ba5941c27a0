#!/usr/bin/env python3
"""VALU roofline inputs for bench.py, from rocprofv3 counters.

  cost:   per-opcode SIMD issue cost from a counter pass over
          ntt-gpu-qtesla_amd/bin/valu_cost (tools/valu_cost.hip):
            python tools/valu_summary.py cost PMC.csv [--out profiles/valu_issue_cost.json]
          cost[op] = SIMD-cycles per wave-instruction
                   = (GRBM_GUI_ACTIVE / 8 XCDs) * 4 SIMDs * CUs / SQ_INSTS_VALU,
          i.e. counted in the cycles the chip actually ran (whatever clock
          DVFS held), not in wall time at an assumed clock.

  kernel: VALU issue demand of one bench workload's dominant kernel, added to
          its profiles/pmc_summary.json entry (stamped with the build hash):
            python tools/valu_summary.py kernel PMC.csv --config 4 [--op/--param/--batch/--ring]
          The counter pass gives SQ_INSTS_VALU and GRBM_GUI_ACTIVE per launch
          (median over launches); the kernel's static opcode mix (tools/
          asm_hist.py over `make asm`) weighted by the cost table gives the mean
          SIMD-cycles per VALU instruction; their product is the VALU issue
          time per launch in SIMD-cycles.  bench.py divides it by the live
          launch time: achieved SIMD-cycles/s against 4 SIMDs x CUs x 2.4 GHz
          (peak) and against the clock the counter pass measured.
"""
import argparse
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ntt-gpu-qtesla_amd"), os.path.join(ROOT, "tools")]
COST_PATH = os.path.join(ROOT, "profiles", "valu_issue_cost.json")
PMC_PATH = os.path.join(ROOT, "profiles", "pmc_summary.json")
XCDS = 8
SIMDS = 4


def load(path):
    """{kernel name: [{counter: value, "ns": duration} per dispatch]}"""
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = rows[(r["Kernel_Name"], int(r["Dispatch_Id"]))]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = defaultdict(list)
    for (k, _), d in sorted(rows.items(), key=lambda x: x[0][1]):
        out[k].append(d)
    return out


def norm_op(op):
    """v_add_u32_e32 / v_add_u32_e64 / v_add_u32 -> v_add_u32"""
    for suf in ("_e32", "_e64", "_sdwa", "_dpp"):
        if op.endswith(suf):
            return op[: -len(suf)]
    return op


def cmd_cost(args):
    import re
    data = load(args.csv)
    cus = args.cus
    table, clocks = {}, []
    for k, ds in data.items():
        m = re.search(r"k_(v_\w+?)\(", k) or re.search(r"k_(v_\w+)", k)
        if not m:
            continue
        d = max(ds, key=lambda x: x.get("SQ_INSTS_VALU", 0))   # the long launch (the other is the warm-up)
        cyc = d["GRBM_GUI_ACTIVE"] / XCDS
        table[m.group(1)] = round(cyc * SIMDS * cus / d["SQ_INSTS_VALU"], 3)
        clocks.append(cyc / d["ns"])
    note = None
    if "v_cndmask_b32_sgpr" in table and "v_cndmask_b32" in table:
        # the compiler's form reads its condition from an SGPR pair nothing in
        # the loop writes; the K32 form clobbers vcc in every asm statement
        table["v_cndmask_b32_vcc_clobber"] = table["v_cndmask_b32"]
        table["v_cndmask_b32"] = table["v_cndmask_b32_sgpr"]
        note = ("v_cndmask_b32: the form with its condition in an SGPR pair nothing writes in the loop (the "
                "compiler's form); the vcc-clobbering form of tools/valu_cost.hip is kept as "
                "v_cndmask_b32_vcc_clobber, an artefact of the test")
    out = {"unit": "SIMD-cycles per wave64 instruction (issue throughput, 8 waves/SIMD, independent chains)",
           "source": os.path.relpath(args.csv, ROOT), "cus": cus,
           "clock_ghz_held": round(statistics.median(clocks), 3), "cost": dict(sorted(table.items()))}
    if note:
        out["note"] = note
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


def mean_cost(hist, cost):
    """mean SIMD-cycles per VALU instruction of a static opcode histogram;
    opcodes without a measured cost count at the v_add_u32 cost (and are
    listed)"""
    tot = w = 0.0
    missing = {}
    base = cost["v_add_u32"]
    for op, k in hist.items():
        c = cost.get(norm_op(op))
        if c is None:
            missing[op] = k
            c = base
        tot += k
        w += k * c
    return w / tot, missing, tot


def cmd_kernel(args):
    import asm_hist
    import bench
    import ntt_amd
    import pmc_summary
    cost = json.load(open(COST_PATH))["cost"]
    c_op, c_param, c_batch, c_ring = bench.CONFIGS[args.config]
    op, param, batch, ring = args.op or c_op, args.param or c_param, args.batch or c_batch, args.ring or c_ring
    info = ntt_amd.param_info(param)
    ps = ntt_amd.PARAM_SETS[param]
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    pats = pmc_summary.kernel_patterns(op, ps, ring)
    data = load(args.csv)
    build = ntt_amd.build_hash()
    summ = json.load(open(args.pmc))
    entry = summ["entries"].get(workload)
    if entry is None:
        sys.exit(f"no PMC entry for {workload}: run tools/pmc_summary.py first")
    if entry.get("build_hash") != build:
        sys.exit(f"PMC entry of {workload} is build {entry.get('build_hash')}, the library is {build}")
    res = {}
    for key, pat in pats.items():
        ds = [d for k, v in data.items() if pat in k for d in v]
        if not ds:
            continue
        insts = statistics.median(d["SQ_INSTS_VALU"] for d in ds)
        cyc = statistics.median(d["GRBM_GUI_ACTIVE"] / XCDS for d in ds)
        clock = statistics.median(d["GRBM_GUI_ACTIVE"] / XCDS / d["ns"] for d in ds)
        # static mix of the kernel (mangled name contains the demangled pieces)
        src = "nussbaumer.s" if "nussbaumer" in pat else "ntt_kernels.s"
        hists = asm_hist.hist(os.path.join(ROOT, "ntt-gpu-qtesla_amd", "build", src), *mangled_parts(pat))
        if len(hists) != 1:
            sys.exit(f"{pat}: {len(hists)} kernels match in build/{src} (run make asm)")
        hist = next(iter(hists.values()))
        c_mean, missing, static_n = mean_cost(hist, cost)
        simd_cyc = insts * c_mean
        res[key] = {"kernel": pat, "launches": len(ds), "SQ_INSTS_VALU": insts, "GRBM_GUI_ACTIVE_per_xcd": cyc,
                    "clock_ghz_pmc": round(clock, 4), "static_valu_per_wave_loop": static_n,
                    "mean_simd_cycles_per_valu": round(c_mean, 4), "valu_simd_cycles_per_launch": simd_cyc,
                    "valu_busy_at_pmc_clock": simd_cyc / (SIMDS * args.cus * cyc),
                    "uncosted_opcodes": missing}
    if not res:
        sys.exit(f"no {op} kernel in {args.csv}")
    entry["valu"] = {"cost_table": os.path.relpath(COST_PATH, ROOT), "cus": args.cus, "source": os.path.relpath(args.csv, ROOT),
                     "kernels": res}
    json.dump(summ, open(args.pmc, "w"), indent=1)
    print(json.dumps(entry["valu"], indent=1))


def mangled_parts(pat):
    """'k_poly_mul<2, false, 0>' -> ('10k_poly_mul', 'ILi2ELb0ELi0E') for the mangled asm label"""
    name, _, targs = pat.partition("<")
    parts = [f"{len(name)}{name}"]
    enc = ""
    for a in targs.rstrip(">").split(","):
        a = a.strip()
        enc += "Lb1E" if a == "true" else "Lb0E" if a == "false" else f"Li{a}E"
    if enc:
        parts.append("I" + enc)
    return tuple(parts)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("cost")
    a.add_argument("csv")
    a.add_argument("--cus", type=int, default=256)
    a.add_argument("--out", default=COST_PATH)
    b = sub.add_parser("kernel")
    b.add_argument("csv")
    b.add_argument("--config", type=int, default=4)
    b.add_argument("--op")
    b.add_argument("--param")
    b.add_argument("--batch", type=int)
    b.add_argument("--ring")
    b.add_argument("--cus", type=int, default=256)
    b.add_argument("--pmc", default=PMC_PATH, help="PMC summary to add the entry to")
    args = ap.parse_args()
    (cmd_cost if args.cmd == "cost" else cmd_kernel)(args)


if __name__ == "__main__":
    main()
