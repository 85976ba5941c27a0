"""bench.py bookkeeping on the CPU: every BASELINE config and the large-n
lines name a workload whose committed PMC traffic entry (profiles/
pmc_summary.json) was measured on the library build in this tree, so the
bench line reports `traffic` instead of null."""
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
def test_pmc_entry_matches_this_build(ntt, op, param, batch, ring):
    info = ntt.param_info(param)
    workload = bench.workload_name(op, param, info["n"], info["q"], ring)
    traffic, note = bench.load_pmc(workload, batch, ntt.build_hash())
    assert traffic is not None, note
    alg = batch * info["n"] * (12 if op in ("polymul", "polymul_ntt", "nussbaumer") else 8)
    assert 0.99 * alg < traffic < 1.1 * alg, (traffic, alg)
