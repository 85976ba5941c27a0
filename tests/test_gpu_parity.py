"""GPU parity: the HIP kernels (through the C ABI) vs the CPU oracle, bit-exact.

Oracle = C restatement of the reference NTT.cu (oracle/ntt_oracle.c), itself
pinned by the constants.h hashes, round-trip identity, the all-ones KAT and
O(n^2) definitions (tests/test_oracle.py).
"""
import numpy as np
import pytest
import torch

from conftest import LARGE_SETS, PARAM_SETS

pytestmark = pytest.mark.gpu


def _u32(ntt, t):
    return ntt.to_numpy_u32(t)


def _dev(ntt, a, dev):
    return ntt.from_numpy_u32(a, dev)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_golden_vectors(ntt, oracle, dev, ps):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"vectors_{ps}.npz"))
    t = _dev(ntt, g["x"], dev)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t), g["X"])
    t = _dev(ntt, g["Xin"], dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), g["xinv"])
    a, b = _dev(ntt, g["x"], dev), _dev(ntt, g["y"], dev)
    c = torch.empty_like(a)
    ntt.poly_mul(c, a, b, ps)
    assert np.array_equal(_u32(ntt, c), g["c"])
    t = _dev(ntt, g["pattern"][None, :], dev)   # init_operand pattern (NTT.cu:10-15)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t)[0], g["pattern_X"])
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t)[0], g["pattern"])


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 2, 3, 64, 257, 8195])
def test_fwd_inv_random(ntt, oracle, dev, ps, batch):
    x = oracle.fill_uniform(batch, ps, 0xC0FFEE + batch, 0)
    t = _dev(ntt, x, dev)
    ntt.poly_ntt(t, ps)
    X = _u32(ntt, t)
    assert np.array_equal(X, oracle.poly_ntt(x, ps))
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), x)
    # inverse of an arbitrary frequency-domain vector
    Y = oracle.fill_uniform(batch, ps, 0xBEEF + batch, 0)
    t = _dev(ntt, Y, dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_invntt(Y, ps))


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 3, 130, 2100])   # 2100: past the latency kernels' 2^21 coefficients
def test_bitrev_order_transforms(ntt, oracle, dev, ps, batch):
    """poly_ntt_bitrev / poly_invntt_bitrev: the NTT domain in bit-reversed order,
    as the reference's CT-CT pipeline keeps it (bit_reverse_copy_tbl_gpu +
    radix2INTT_gpu0/1/2 on bit-reversed input, NTT.cu:2239-2249)."""
    br = ntt.tables(ps)["bitrev_tbl"]
    x = oracle.fill_uniform(batch, ps, 0xB17 + batch, 0)
    X = oracle.poly_ntt(x, ps)
    tx = _dev(ntt, x, dev)
    o = torch.empty_like(tx)
    ntt.poly_ntt_bitrev(o, tx, ps)
    assert np.array_equal(_u32(ntt, o), X[:, br])
    assert np.array_equal(_u32(ntt, tx), x)            # out of place keeps the input
    ntt.poly_invntt_bitrev(tx, o, ps)
    assert np.array_equal(_u32(ntt, tx), x)
    # inverse of an arbitrary bit-reversed-order vector vs the oracle's CT-CT inverse
    Ybr = oracle.fill_uniform(batch, ps, 0xB18 + batch, 0)
    want = oracle.poly_invntt_ct(oracle.bit_reverse_copy(Ybr, ps), ps)
    assert np.array_equal(want, oracle.poly_invntt(Ybr[:, br], ps))
    t = _dev(ntt, Ybr, dev)
    ntt.poly_invntt_bitrev(t, t, ps)                     # in place
    assert np.array_equal(_u32(ntt, t), want)
    # the CT-CT composition: bitrev copy then the bit-reversed inverse == poly_invntt
    t = _dev(ntt, X, dev)
    ntt.poly_bitrev_copy(t, t, ps)
    ntt.poly_invntt_bitrev(t, t, ps)
    assert np.array_equal(_u32(ntt, t), x)


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [33, 2100])   # latency kernels / batch kernels
def test_out_of_place_keeps_input(ntt, oracle, dev, ps, batch):
    x = oracle.fill_uniform(batch, ps, 7, 0)
    tin = _dev(ntt, x, dev)
    tout = torch.empty_like(tin)
    ntt.poly_ntt_oop(tout, tin, ps)
    assert np.array_equal(_u32(ntt, tin), x)          # unlike NTT.cu:506, input kept
    assert np.array_equal(_u32(ntt, tout), oracle.poly_ntt(x, ps))
    back = torch.empty_like(tin)
    ntt.poly_invntt_oop(back, tout, ps)
    assert np.array_equal(_u32(ntt, back), x)


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 5, 128, 2100])   # 2100: past the latency kernels' 2^21 coefficients
def test_poly_mul_random(ntt, oracle, dev, ps, batch):
    a = oracle.fill_uniform(batch, ps, 11 + batch, 0)
    b = oracle.fill_uniform(batch, ps, 12 + batch, 0)
    ta, tb = _dev(ntt, a, dev), _dev(ntt, b, dev)
    tc = torch.empty_like(ta)
    ntt.poly_mul(tc, ta, tb, ps)
    want = oracle.poly_mul(a, b, ps)
    assert np.array_equal(_u32(ntt, tc), want)
    assert np.array_equal(want[0], oracle.schoolbook_np(a[0], b[0], ps))
    # aliasing output with an input is allowed
    ntt.poly_mul(ta, ta, tb, ps)
    assert np.array_equal(_u32(ntt, ta), want)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_reference_pipelines_kat(ntt, oracle, dev, ps):
    """All-ones operands of the reference drivers (NTT.cu:2360): z[k] = 2k+2-n mod q."""
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    ones = np.ones((2, n), np.uint32)   # BATCH = 2 (main.cuh:7)
    want = ((2 * np.arange(n) + 2 - n) % q).astype(np.uint32)
    ta, tb = _dev(ntt, ones, dev), _dev(ntt, ones, dev)
    tc = torch.empty_like(ta)
    ntt.poly_mul(tc, ta, tb, ps)
    assert all(np.array_equal(r, want) for r in _u32(ntt, tc))
    # composed CT-GS pipeline through the individual entry points
    ntt.poly_ntt(ta, ps)
    ntt.poly_ntt(tb, ps)
    ntt.poly_pointwise(tc, ta, tb, ps)
    ntt.poly_invntt(tc, ps)
    assert all(np.array_equal(r, want) for r in _u32(ntt, tc))
    # and the reference's own GPU kernel order, restated in the oracle
    assert np.array_equal(oracle.gpu_ct_gs_polymul(ones, ones, ps)[0], want)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_pointwise(ntt, oracle, dev, ps):
    a = oracle.fill_uniform(9, ps, 21, 0)
    b = oracle.fill_uniform(9, ps, 22, 0)
    ta, tb = _dev(ntt, a, dev), _dev(ntt, b, dev)
    tc = torch.empty_like(ta)
    ntt.poly_pointwise(tc, ta, tb, ps)
    assert np.array_equal(_u32(ntt, tc), oracle.pointwise(a, b, ps).reshape(a.shape))


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("reps", [1, 420])   # 5 / 2100 polynomials: latency kernels / batch kernels
def test_edge_values(ntt, oracle, dev, ps, reps):
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    cases = np.stack([np.zeros(n, np.uint32), np.full(n, q - 1, np.uint32),
                      np.eye(1, n, 0, dtype=np.uint32)[0], np.eye(1, n, n - 1, dtype=np.uint32)[0],
                      (np.arange(n) % 2 * (q - 1)).astype(np.uint32)])
    cases = np.tile(cases, (reps, 1))
    t = _dev(ntt, cases, dev)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_ntt(cases, ps))
    t = _dev(ntt, cases, dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_invntt(cases, ps))
    tc = torch.empty_like(t)
    ta = _dev(ntt, cases, dev)
    ntt.poly_mul(tc, ta, ta, ps)
    assert np.array_equal(_u32(ntt, tc), oracle.poly_mul(cases, cases, ps))


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [4, 2100])   # latency kernels / batch kernels
def test_lazy_inputs_below_2q(ntt, oracle, dev, ps, batch):
    """Inputs in [q, 2q) are tolerated: result == transform of (input mod q)."""
    q = ntt.param_info(ps)["q"]
    x = oracle.fill_uniform(batch, ps, 99, 0)
    xl = (x.astype(np.uint64) + q).astype(np.uint32)
    t = _dev(ntt, xl, dev)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_ntt(x, ps))
    t = _dev(ntt, xl, dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_invntt(x, ps))


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_fill_uniform_matches_host_generator(ntt, oracle, dev, ps):
    n = ntt.param_info(ps)["n"]
    t = torch.empty(6 * n, dtype=torch.int32, device=dev)
    ntt.fill_uniform(t, ps, 0x1234, first_poly=1000)
    assert np.array_equal(_u32(ntt, t).reshape(6, n), oracle.fill_uniform(6, ps, 0x1234, 1000))


def test_batch_zero_and_errors(ntt, dev):
    t = torch.zeros(2048, dtype=torch.int32, device=dev)
    assert ntt.lib().poly_ntt(t.data_ptr(), None, 0, 2, None) == 0
    assert ntt.lib().poly_ntt(t.data_ptr(), None, 1, 7, None) == ntt.NTT_ERR_PARAM
    assert ntt.lib().poly_ntt(t.data_ptr() + 2, None, 1, 2, None) == ntt.NTT_ERR_ALIGN
    with pytest.raises(ntt.NTTError):
        ntt.poly_ntt(t, 9)


def test_device_checks(ntt, dev):
    """Operands on different devices are rejected; a tensor on a non-current
    device runs on its own device and stream."""
    n = 2048
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        ntt.poly_mul(a, a, torch.zeros(n, dtype=torch.int32), "p-III")
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: the non-current-device case needs two")
    other = torch.device("cuda", 1)
    b = torch.ones(n, dtype=torch.int32, device=other)
    with pytest.raises(ValueError):
        ntt.poly_mul(a, a, b, "p-III")
    with torch.cuda.device(0):
        ntt.poly_ntt(b, "p-III")
        ntt.poly_invntt(b, "p-III")
    torch.cuda.synchronize(other)
    assert torch.equal(b.cpu(), torch.ones(n, dtype=torch.int32))


def test_nondefault_stream(ntt, oracle, dev):
    ps = "p-III"
    x = oracle.fill_uniform(50, ps, 5, 0)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        t = _dev(ntt, x, dev)
        ntt.poly_ntt(t, ps, s)
        ntt.poly_invntt(t, ps, s)
    s.synchronize()
    assert np.array_equal(_u32(ntt, t), x)


@pytest.mark.slow
@pytest.mark.parametrize("ps,batch", [("p-III", 1 << 20), ("p-I", 65536), ("ref", 65536), ("p-III", 300001)])
def test_full_batch_properties(ntt, oracle, dev, ps, batch):
    """BASELINE sizes: round trip on the whole batch on device + sampled polys vs oracle."""
    n = ntt.param_info(ps)["n"]
    x = torch.empty(batch * n, dtype=torch.int32, device=dev)
    ntt.fill_uniform(x, ps, 0x5EED0003, 0)
    ref = x.clone()
    ntt.poly_ntt(x, ps)
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([[0, batch - 1], rng.integers(0, batch, 254)]))
    X = x.view(batch, n)[torch.as_tensor(idx, device=dev)]
    xs = ntt.to_numpy_u32(ref.view(batch, n)[torch.as_tensor(idx, device=dev)])
    assert np.array_equal(ntt.to_numpy_u32(X), oracle.poly_ntt(xs, ps))
    ntt.poly_invntt(x, ps)
    assert torch.equal(x, ref)
    # linearity on the whole batch, on device: NTT(a) + NTT(b) == NTT(a + b mod q)
    q = ntt.param_info(ps)["q"]
    b = torch.empty_like(x)
    ntt.fill_uniform(b, ps, 0x5EED0004, 0)
    s = ((ref.to(torch.int64) & 0xFFFFFFFF) + (b.to(torch.int64) & 0xFFFFFFFF)) % q
    s = s.to(torch.int32)
    del ref
    ntt.poly_ntt(x, ps)
    ntt.poly_ntt(b, ps)
    ntt.poly_ntt(s, ps)
    lhs = ((x.to(torch.int64) & 0xFFFFFFFF) + (b.to(torch.int64) & 0xFFFFFFFF)) % q
    assert torch.equal(lhs, s.to(torch.int64) & 0xFFFFFFFF)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_host_driver_kat(ps):
    """The C++ host driver (reference CLI) reports the all-ones KAT as Identical."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ntt-gpu-qtesla_amd", "bin", "ntt_main")
    for opt in ("6", "7"):
        r = subprocess.run([exe, "-speedgpu", opt, "-param", ps, "-batch", "4"], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert "Identical." in r.stdout, r.stdout
    r = subprocess.run([exe, "-speedgpu", "9", "-param", ps, "-batch", "1000", "-r", "5"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "Identical." in r.stdout, r.stdout + r.stderr
    for opt, batch in (("10", "5000"), ("11", "7")):   # host pipeline (2 chunks at n=1024), Nussbaumer mod 2^32-1
        r = subprocess.run([exe, "-speedgpu", opt, "-param", ps, "-batch", batch], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0 and "Identical." in r.stdout, r.stdout + r.stderr
    # per-call latency option: one JSON line per entry point, small batch
    r = subprocess.run([exe, "-speedgpu", "12", "-param", ps, "-batch", "1", "-reps", "50"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [d["op"] for d in lines] == ["poly_ntt", "poly_invntt", "poly_mul"]
    assert all(0 < d["back_to_back_us"] < 1e4 and d["calls"] == 50 for d in lines)


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 3, 64, 2100])
def test_poly_mul_ntt_domain(ntt, oracle, dev, ps, batch):
    """poly_mul_ntt(c, a, poly_ntt(b)) == a*b mod (x^n+1, q): the CT-GS driver
    with b's forward transform done beforehand (qTESLA's NTT-domain operand)."""
    a = oracle.fill_uniform(batch, ps, 41 + batch, 0)
    b = oracle.fill_uniform(batch, ps, 42 + batch, 0)
    want = oracle.poly_mul(a, b, ps)
    ta = _dev(ntt, a, dev)
    tb = _dev(ntt, oracle.poly_ntt(b, ps), dev)
    tc = torch.empty_like(ta)
    ntt.poly_mul_ntt(tc, ta, tb, ps)
    assert np.array_equal(_u32(ntt, tc), want)
    # b-hat entries in [q, 2q) are tolerated; aliasing c with a is allowed
    q = ntt.param_info(ps)["q"]
    bl = (oracle.poly_ntt(b, ps).astype(np.uint64) + q).astype(np.uint32)
    ntt.poly_mul_ntt(ta, ta, _dev(ntt, bl, dev), ps)
    assert np.array_equal(_u32(ntt, ta), want)


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 3, 130])
def test_bitrev_copy(ntt, oracle, dev, ps, batch):
    """poly_bitrev_copy == bit_reverse_copy_tbl_gpu (NTT.cu:487-492) on arbitrary 32-bit words."""
    n = ntt.param_info(ps)["n"]
    rng = np.random.default_rng(batch + n)
    x = rng.integers(0, 1 << 32, (batch, n), dtype=np.uint64).astype(np.uint32)
    want = x[:, ntt.tables(ps)["bitrev_tbl"]]
    assert np.array_equal(want, oracle.bit_reverse_copy(x, ps))
    t = _dev(ntt, x, dev)
    o = torch.empty_like(t)
    ntt.poly_bitrev_copy(o, t, ps)
    assert np.array_equal(_u32(ntt, o), want)
    ntt.poly_bitrev_copy(t, t, ps)          # in place
    assert np.array_equal(_u32(ntt, t), want)


# switch points above this batch are not tested (an in-place n = 1024
# transform takes the radix-16 kernels for every batch the ABI accepts)
MAX_TEST_BATCH = 1 << 20


def _switch_points(ntt, ps, op):
    """Every batch at which entry point `op` changes kernel family
    (ntt_small_batch_radix: radix-4 / 8 / 16 one-polynomial-per-workgroup
    tiers, then the batch kernels), found by bisection: the last batch of each
    tier and the first of the next."""
    m = ntt.small_batch_max(ps, op)
    pts = []
    lo = 1
    while lo <= m and lo < MAX_TEST_BATCH:
        r = ntt.small_batch_radix(ps, op, lo)
        a, b = lo, m + 1          # radix(a) == r, radix(b) != r
        while b - a > 1:
            mid = (a + b) // 2
            if ntt.small_batch_radix(ps, op, mid) == r:
                a = mid
            else:
                b = mid
        pts += [a, b]
        lo = b
    return sorted(p for p in set(pts) if p <= MAX_TEST_BATCH)


@pytest.mark.parametrize("ps", PARAM_SETS + LARGE_SETS)
@pytest.mark.parametrize("op", ["fwd", "inv", "fwd_br", "inv_br", "mul", "mul_ntt", "fwd_oop", "inv_oop"])
def test_latency_switch_boundary(ntt, oracle, dev, ps, op):
    """On both sides of every switch point of this entry point (the tiers of
    csrc/ntt_lat.hpp: radix-4 / 8 / 16 one-polynomial-per-workgroup kernels,
    then the batch kernels) the results equal the oracle's.  Inputs come from
    the device generator; 40 sampled polynomials of each launch (first, last,
    random) are regenerated on the host and checked."""
    if ntt.small_batch_max(ps, op) == 0:
        pytest.skip("no small-batch kernel for this entry point")
    n = ntt.param_info(ps)["n"]
    brv = ntt.tables(ps)["bitrev_tbl"]
    for batch in _switch_points(ntt, ps, op):
        rows = sorted({0, 1, batch // 2, batch - 2, batch - 1} |
                      set(np.random.default_rng(batch).integers(0, batch, 35).tolist()))
        rows = [r for r in rows if 0 <= r < batch]
        ri = torch.tensor(rows, device=dev)
        seed = 0x51DE + batch
        tx = torch.empty(batch * n, dtype=torch.int32, device=dev)
        ntt.fill_uniform(tx, ps, seed)
        xs = np.concatenate([oracle.fill_uniform(1, ps, seed, r) for r in rows])
        tz = torch.empty_like(tx)
        got = lambda t: _u32(ntt, t.view(batch, n)[ri])   # noqa: E731
        if op == "fwd":
            ntt.poly_ntt(tx, ps)
            assert np.array_equal(got(tx), oracle.poly_ntt(xs, ps)), batch
        elif op == "inv":
            ntt.poly_invntt(tx, ps)
            assert np.array_equal(got(tx), oracle.poly_invntt(xs, ps)), batch
        elif op == "fwd_oop":
            ntt.poly_ntt_oop(tz, tx, ps)
            assert np.array_equal(got(tz), oracle.poly_ntt(xs, ps)), batch
        elif op == "inv_oop":
            ntt.poly_invntt_oop(tz, tx, ps)
            assert np.array_equal(got(tz), oracle.poly_invntt(xs, ps)), batch
        elif op == "fwd_br":
            ntt.poly_ntt_bitrev(tz, tx, ps)
            assert np.array_equal(got(tz), oracle.poly_ntt(xs, ps)[:, brv]), batch
        elif op == "inv_br":
            ntt.poly_invntt_bitrev(tz, tx, ps)
            assert np.array_equal(got(tz), oracle.poly_invntt(xs[:, brv], ps)), batch
        else:
            ty = torch.empty_like(tx)
            ntt.fill_uniform(ty, ps, seed + 1)
            ys = np.concatenate([oracle.fill_uniform(1, ps, seed + 1, r) for r in rows])
            want = oracle.poly_mul(xs, ys, ps)
            if op == "mul":
                ntt.poly_mul(tz, tx, ty, ps)
            else:
                ntt.poly_ntt(ty, ps)   # b-hat; verified by the "fwd" case
                ntt.poly_mul_ntt(tz, tx, ty, ps)
            assert np.array_equal(got(tz), want), batch
