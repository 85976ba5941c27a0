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
