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


def test_load_pmc_reports_stale_build(ntt):
    """A hash mismatch yields traffic None plus the reason, never a stale number."""
    op, param, batch, ring = bench.CONFIGS[3]
    info = ntt.param_info(param)
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    traffic, note = bench.load_pmc(workload, batch, "0000000000000000")
    assert traffic is None and "this library is 0000000000000000" in note
