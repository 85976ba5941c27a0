"""Build identity of the product library (CPU only, no GPU calls).

bench.py ties the committed PMC traffic / VALU entries (profiles/
pmc_summary.json) to the library they were measured on through the
Makefile's SRC_HASH ("src=" in ntt_build_info).  That tie only holds if the
hash covers every file the product translation units include, and `make`
only rebuilds a stale library if the same list is its prerequisite list.
These tests take the compiler's own dependency scan (hipcc -MM) as the truth.
"""
import hashlib
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ntt-gpu-qtesla_amd")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _make_vars():
    out = subprocess.run(["make", "-s", "-n", "-p", "-C", PKG], capture_output=True, text=True).stdout
    v = {}
    for line in out.splitlines():
        for name in ("SRCS", "HDRS", "SRC_HASH", "HIPFLAGS", "ARCH"):
            if line.startswith(name + " := ") or line.startswith(name + " = "):
                v[name] = line.split("=", 1)[1].strip()
    return v


def _norm(p):
    return os.path.normpath(os.path.join(PKG, p))


@pytest.fixture(scope="module")
def mk():
    v = _make_vars()
    for k in ("SRCS", "HDRS", "SRC_HASH"):
        assert k in v, f"make -p did not report {k}"
    return v


@pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"), reason="no hipcc")
def test_every_included_file_is_hashed(mk):
    """Every in-tree file in the -MM dependency list of the product TUs is in
    the Makefile's HDRS/SRCS (so it is hashed into src= and is a rebuild
    prerequisite of lib/libqtesla_ntt.so)."""
    srcs = mk["SRCS"].split()
    r = subprocess.run([HIPCC, "-std=c++17", "--offload-arch=gfx950", "--cuda-host-only", "-MM", *srcs],
                       capture_output=True, text=True, cwd=PKG)
    assert r.returncode == 0, r.stderr
    deps = set()
    for tok in r.stdout.replace("\\\n", " ").split():
        if tok.endswith(":"):
            continue
        path = _norm(tok)
        if path.startswith(ROOT + os.sep):
            deps.add(path)
    hashed = {_norm(p) for p in mk["SRCS"].split() + mk["HDRS"].split()}
    missing = sorted(os.path.relpath(p, ROOT) for p in deps - hashed)
    assert not missing, f"included by the product TUs but not hashed / not a prerequisite: {missing}"
    # the large-n kernels' header in particular
    assert _norm("csrc/ntt_big.hpp") in hashed


def test_src_hash_recomputes(mk):
    """SRC_HASH = sha256(HIPFLAGS ARCH + the text of SRCS then HDRS)[:16]."""
    h = hashlib.sha256()
    flags = mk.get("HIPFLAGS", "").replace("$(ARCH)", mk.get("ARCH", ""))   # make -p prints it unexpanded
    h.update(f"{flags} {mk.get('ARCH', '')}\n".encode())
    for p in mk["SRCS"].split() + mk["HDRS"].split():
        with open(_norm(p), "rb") as f:
            h.update(f.read())
    assert h.hexdigest()[:16] == mk["SRC_HASH"]


@pytest.mark.parametrize("hdr", ["csrc/ntt_big.hpp", "csrc/ntt_large.hpp", "csrc/ntt_device.hpp", "csrc/pset.hpp"])
def test_header_edit_schedules_rebuild(hdr):
    """`make -n -W <header> lib/libqtesla_ntt.so` schedules the library's
    compile: an edit to any product header rebuilds it."""
    r = subprocess.run(["make", "-n", "-C", PKG, "-W", hdr, "lib/libqtesla_ntt.so"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "-shared -o lib/libqtesla_ntt.so" in r.stdout, r.stdout
