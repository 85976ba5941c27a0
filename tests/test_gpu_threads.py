"""Reentrancy of the C ABI across host threads and streams (include/
qtesla_ntt.h: "reentrant across streams and devices"): concurrent FIRST
calls from several host threads of a fresh process -- the per-device table
upload happens exactly once while the others wait, later calls take the
lock-free path -- then interleaved launches on distinct streams, every
thread's results bit-exact against the oracle (tests/thread_worker.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nthreads", [4, 8])
def test_concurrent_first_calls_on_distinct_streams(ntt, oracle, nthreads):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "thread_worker.py"), str(nthreads)],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert len(res["threads"]) == nthreads
    for t in res["threads"]:
        assert t["rc_ok"] and t["ntt"] and t["mul"], t
    assert res["expiries"] == 0
