"""bench.py bookkeeping on the CPU: every BASELINE config and the large-n
lines name a workload that has a committed PMC traffic entry (profiles/
pmc_summary.json) with a sane traffic / algorithmic-bytes ratio.  Whether
the entry was measured on the library build in this tree is bench.py's
business at run time (it reports `traffic: null` with the reason when the
build hash differs), so an ordinary source edit does not fail this suite."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _cases():
    for c, (op, param, batch, ring) in sorted(bench.CONFIGS.items()):
        if c == 1:
            continue   # batch-1 latency line: no PMC pass (traffic is meaningless there)
        yield op, param, batch, ring
    for n in (4096, 8192):
        yield "fwdinv", f"p-III-{n}", (1 << 33) // 4 // n, "q"


@pytest.mark.parametrize("op,param,batch,ring", list(_cases()))
def test_pmc_entry_sane(ntt, op, param, batch, ring):
    info = ntt.param_info(param)
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    with open(bench.PMC_PATH) as f:
        entries = json.load(f)["entries"]
    e = entries.get(workload)
    assert e is not None, f"no PMC entry for {workload}"
    assert e["batch"] == batch
    assert isinstance(e.get("build_hash"), str) and len(e["build_hash"]) == 16
    alg = batch * info["n"] * (12 if op in ("polymul", "polymul_ntt", "nussbaumer") else 8)
    assert 0.99 * alg < e["hbm_bytes_per_launch"] < 1.1 * alg, (e["hbm_bytes_per_launch"], alg)


def _tree_hash():
    """SRC_HASH of the sources in this tree, as the Makefile computes it."""
    import subprocess
    out = subprocess.run(["make", "-s", "-n", "-p", "-C", os.path.join(ROOT, "ntt-gpu-qtesla_amd")],
                         capture_output=True, text=True).stdout
    for line in out.splitlines():
        if line.startswith("SRC_HASH := ") and len(line.split()[-1]) == 16:
            return line.split()[-1]
    return None


def test_pmc_summary_matches_tree_build():
    """Non-blocking staleness check: the committed PMC summary should have been
    measured on the library these sources build.  A source edit without a new
    measurement xfails here (bench.py then reports traffic: null)."""
    with open(bench.PMC_PATH) as f:
        entries = json.load(f)["entries"]
    tree = _tree_hash()
    if tree is None:
        pytest.skip("make -p did not report SRC_HASH")
    stale = sorted({e.get("build_hash") for e in entries.values()} - {tree})
    if stale:
        pytest.xfail(f"profiles/pmc_summary.json measured on build(s) {stale}, the tree builds {tree}")


def test_load_pmc_reports_stale_build(ntt):
    """A hash mismatch yields traffic None plus the reason, never a stale number."""
    op, param, batch, ring = bench.CONFIGS[3]
    info = ntt.param_info(param)
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    traffic, note = bench.load_pmc(workload, batch, "0000000000000000")
    assert traffic is None and "this library is 0000000000000000" in note


def test_valu_roofline_fields():
    """VALU-bound ops report roofline.bound "valu": SIMD issue cycles per
    launch (SQ_INSTS_VALU x mean opcode cost) over the live launch time,
    against 4 SIMDs x CUs x 2.4 GHz, with the HBM fraction kept beside it.
    The held-clock fraction comes from the counter pass alone (its busy value),
    whatever this run's launch time is."""
    v = {"valu_simd_cycles_per_launch": 1024 * 2.4e9 * 5e-3, "clock_ghz_pmc": 2.0, "cus": 256,
         "SQ_INSTS_VALU": 1.0, "mean_simd_cycles_per_valu": 3.5, "valu_busy_at_pmc_clock": 0.87,
         "uncosted_opcodes": {}}
    r = bench.valu_roofline(v, 10.0, {"bound": "hbm", "frac": 0.4})
    assert r["bound"] == "valu" and r["unit"] == "G SIMD-cycles/s"
    assert abs(r["frac"] - 0.5) < 1e-12 and r["frac_at_held_clock"] == 0.87
    assert bench.valu_roofline(v, 7.0, {})["frac_at_held_clock"] == 0.87   # independent of the live time
    assert r["hbm"]["frac"] == 0.4
    assert bench.valu_roofline(None, 10.0, {})["frac"] is None
    assert {"polymul", "polymul_ntt", "nussbaumer"} == bench.VALU_BOUND


def _valu_entries():
    with open(bench.PMC_PATH) as f:
        entries = json.load(f)["entries"]
    return {w: e for w, e in entries.items() if "valu" in e}


def test_valu_entries_fully_costed():
    """Every VALU opcode the measured kernels emit has a measured issue cost
    (tools/valu_cost.hip), so the mean cycles per instruction carries no
    guessed term; the held-clock fraction the line reports is the entry's own
    busy value (one counter pass: VALU SIMD-cycles over its GRBM cycles)."""
    ents = _valu_entries()
    assert ents
    tree = _tree_hash()
    if tree is not None and any(e.get("build_hash") != tree for e in ents.values()):
        pytest.xfail("profiles/pmc_summary.json VALU entries were measured on another build")
    for w, e in ents.items():
        for key, k in e["valu"]["kernels"].items():
            assert k["uncosted_opcodes"] == {}, (w, key, k["uncosted_opcodes"])
            busy = k["valu_simd_cycles_per_launch"] / (4 * e["valu"].get("cus", 256) * k["GRBM_GUI_ACTIVE_per_xcd"])
            assert abs(busy - k["valu_busy_at_pmc_clock"]) < 0.01 * busy, (w, key)
            r = bench.valu_roofline(dict(k, cus=e["valu"].get("cus", 256)), 1.0, {})
            assert abs(r["frac_at_held_clock"] - k["valu_busy_at_pmc_clock"]) < 0.01 * k["valu_busy_at_pmc_clock"]


def test_valu_cost_table_classes():
    """The committed issue-cost table (tools/valu_cost.hip under rocprofv3):
    the VOP2 add/sub/logic ops issue at about twice the rate of min/max and
    the multiply class, which is what the poly_mul / Nussbaumer VALU roofline weights by."""
    with open(os.path.join(ROOT, "profiles", "valu_issue_cost.json")) as f:
        cost = json.load(f)["cost"]
    assert cost["v_add_u32"] < 3.0 and cost["v_sub_u32"] < 3.0
    for op in ("v_min_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_i64_i32"):
        assert 4.0 < cost[op] < 5.0, op


@pytest.mark.parametrize("config", [4, 5])
def test_valu_entry_of_valu_bound_configs(ntt, config):
    """The committed PMC summary carries the VALU counter entry the config-4 /
    config-5 lines report as their roofline (tools/valu_summary.py kernel):
    measured on the same build as the traffic, with a busy fraction a
    VALU-bound kernel can have."""
    op, param, batch, ring = bench.CONFIGS[config]
    info = ntt.param_info(param)
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    with open(bench.PMC_PATH) as f:
        e = json.load(f)["entries"][workload]
    assert op in bench.VALU_BOUND
    k = next(iter(e["valu"]["kernels"].values()))
    assert k["SQ_INSTS_VALU"] > 1e9 and 3.0 < k["mean_simd_cycles_per_valu"] < 5.0
    assert 0.5 < k["valu_busy_at_pmc_clock"] < 1.0
    assert 1.5 < k["clock_ghz_pmc"] < 2.5


def test_pattern_floor_skips_non_transforms_and_missing_library(monkeypatch):
    """roofline.pattern_floor_ms is a transform-only diagnostic: product lines
    get none, and a tree without the tools library says so instead of failing."""
    import types
    args = types.SimpleNamespace(op="polymul", param="p-III")
    assert bench.pattern_floor(args, None, None, None, None, 10) is None

    class _N:
        @staticmethod
        def param_info(p):
            return {"n": 2048}
    monkeypatch.setattr(bench, "DIAG_PATH", "/nonexistent/libqtesla_ntt_diag.so")
    args = types.SimpleNamespace(op="fwdinv", param="p-III")
    r = bench.pattern_floor(args, _N, None, None, None, 10)
    assert "not built" in r["note"]
    args = types.SimpleNamespace(op="fwdinv", param="p-III-8192")

    class _N8:
        @staticmethod
        def param_info(p):
            return {"n": 8192}
    # n > 2048: the one-wave kernels' memory-only variant (ntt_diag.hip op 7) is asked for too
    assert "not built" in bench.pattern_floor(args, _N8, None, None, None, 10)["note"]


def test_latency_threshold_matches_kernels(ntt, monkeypatch, tmp_path):
    """bench asks the library which path a batch takes (ntt_small_batch_max /
    ntt_small_batch_radix, csrc/ntt_lat.hpp); on the radix-4 small-batch
    kernels a transform line carries no pattern floor (the diagnostic library
    has no memory-only variant of them)."""
    import types
    monkeypatch.setattr(bench, "DIAG_PATH", str(tmp_path / "diag.so"))
    (tmp_path / "diag.so").write_bytes(b"")
    m = ntt.small_batch_max("p-I", "fwd")
    assert m >= 1
    assert bench.runs_latency_kernels(ntt, "fwd", "p-I", m)
    assert not bench.runs_latency_kernels(ntt, "fwd", "p-I", m + 1)
    assert not bench.runs_latency_kernels(ntt, "nussbaumer", "p-III", 1)
    assert ntt.small_batch_radix("p-I", "fwd", 1) == 4
    x = types.SimpleNamespace(numel=lambda: 1024)
    r = bench.pattern_floor(types.SimpleNamespace(op="fwd", param="p-I"), ntt, None, x, None, 10)
    assert "radix-4" in r["note"]


def test_switch_table_in_library(ntt):
    """ntt_small_batch_max / ntt_small_batch_radix: every (param set, op)
    answers; the tiers only grow the radix-4 -> 8 -> 16 order below the max
    and the batch kernels (0) run above it; the n = 8192 products have no
    small-batch kernel; bad arguments are rejected without a GPU."""
    import ctypes
    for ps in ntt.PARAM_SETS:
        for op in ntt.SWITCH_OPS:
            m = ntt.small_batch_max(ps, op)
            if ntt.param_info(ps)["n"] == 8192 and op.startswith("mul"):
                assert m == 0
                continue
            assert m >= 1, (ps, op)
            assert ntt.small_batch_radix(ps, op, m) in (4, 8, 16)
            assert ntt.small_batch_radix(ps, op, m + 1) == 0
            assert ntt.small_batch_radix(ps, op, 1) in (4, 8, 16)
            if op.startswith("mul"):
                assert ntt.small_batch_radix(ps, op, m) == 4   # the products: radix-4 kernels only
    L = ntt.lib()
    v = ctypes.c_size_t()
    r = ctypes.c_int()
    assert L.ntt_small_batch_max(7, 0, ctypes.byref(v)) == ntt.NTT_ERR_PARAM
    assert L.ntt_small_batch_max(0, 8, ctypes.byref(v)) == ntt.NTT_ERR_PARAM
    assert L.ntt_small_batch_max(0, 0, None) == ntt.NTT_ERR_NULL
    assert L.ntt_small_batch_radix(0, 8, 1, ctypes.byref(r)) == ntt.NTT_ERR_PARAM
    assert L.ntt_small_batch_radix(0, 0, 1, None) == ntt.NTT_ERR_NULL


def test_native_latency_reports_instead_of_raising():
    """The config-1 line's native per-call leg (ntt_main -speedgpu 12 as a
    child process) is a diagnostic: without a GPU (here) it reports why, it
    never raises."""
    import types
    r = bench.native_latency(types.SimpleNamespace(op="fwd", param="p-I"), 1)
    assert ("native_c_abi_us_per_call" in r) or ("native_note" in r)


def test_final_verify_lines_carry_this_builds_counters():
    """The newest round's re-run bench lines (profiles/rNN/final/verify/, run
    after the PMC summary was re-stamped for the measured build) carry the
    counters of their own build: every VALU-bound line with a VALU entry has
    a frac and no note naming another build, every HBM-bound line a traffic
    figure (VERDICT r05 ask 7)."""
    import glob
    import json
    rounds = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "final", "verify")))
    if not rounds:
        pytest.skip("no final/verify lines committed")
    lines = sorted(glob.glob(os.path.join(rounds[-1], "bench*.json")))
    assert lines, rounds[-1]
    hashes = set()
    for f in lines:
        d = json.load(open(f))
        r = d["roofline"]
        hashes.add(d["build"]["hash"])
        note = r.get("valu_note") or r.get("traffic_note") or ""
        assert "measured on build" not in note, (f, note)
        if r["bound"] == "valu":
            if "no VALU counter entry" in note:
                continue   # poly_mul_ntt lines: no counter pass of their own
            assert r["frac"] is not None and r["frac_at_held_clock"] is not None, f
        else:
            assert r["traffic"] is not None, f
    assert len(hashes) == 1, hashes
