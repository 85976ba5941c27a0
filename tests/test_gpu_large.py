"""GPU parity of the n = 4096 / 8192 transforms (multi-wave four-step kernels,
ntt_large.hpp) against the CPU oracle, bit-exact.

The oracle at these sizes is pinned by tests/test_oracle_large.py (O(n^2)
definition, round trip on the reference's operand pattern, all-ones KAT).
"""
import numpy as np
import pytest
import torch

from conftest import LARGE_SETS

pytestmark = pytest.mark.gpu


def _u32(ntt, t):
    return ntt.to_numpy_u32(t)


def _dev(ntt, a, dev):
    return ntt.from_numpy_u32(a, dev)


@pytest.mark.parametrize("ps", LARGE_SETS)
@pytest.mark.parametrize("batch", [1, 2, 3, 7, 64, 1001])
def test_large_fwd_inv_random(ntt, oracle, dev, ps, batch):
    x = oracle.fill_uniform(batch, ps, 0xA11CE + batch, 0)
    t = _dev(ntt, x, dev)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_ntt(x, ps))
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), x)
    Y = oracle.fill_uniform(batch, ps, 0xB0B + batch, 0)
    t = _dev(ntt, Y, dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_invntt(Y, ps))


@pytest.mark.parametrize("ps", LARGE_SETS)
@pytest.mark.parametrize("reps", [1, 100])   # 6 / 600 polynomials: latency kernels / batch kernels
def test_large_edge_values_and_lazy_inputs(ntt, oracle, dev, ps, reps):
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    cases = np.stack([np.zeros(n, np.uint32), np.full(n, q - 1, np.uint32),
                      np.eye(1, n, 0, dtype=np.uint32)[0], np.eye(1, n, n - 1, dtype=np.uint32)[0],
                      np.eye(1, n, n // 2, dtype=np.uint32)[0], (np.arange(n) % 2 * (q - 1)).astype(np.uint32)])
    cases = np.tile(cases, (reps, 1))
    for fwd in (True, False):
        t = _dev(ntt, cases, dev)
        (ntt.poly_ntt if fwd else ntt.poly_invntt)(t, ps)
        want = oracle.poly_ntt(cases, ps) if fwd else oracle.poly_invntt(cases, ps)
        assert np.array_equal(_u32(ntt, t), want)
    x = oracle.fill_uniform(3 * reps, ps, 77, 0)
    xl = (x.astype(np.uint64) + q).astype(np.uint32)   # inputs in [q, 2q)
    t = _dev(ntt, xl, dev)
    ntt.poly_ntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_ntt(x, ps))
    t = _dev(ntt, xl, dev)
    ntt.poly_invntt(t, ps)
    assert np.array_equal(_u32(ntt, t), oracle.poly_invntt(x, ps))


@pytest.mark.parametrize("ps", LARGE_SETS)
@pytest.mark.parametrize("reps", [1, 600])   # latency kernels / batch kernels
def test_large_out_of_place_and_pattern(ntt, oracle, dev, ps, reps):
    n = ntt.param_info(ps)["n"]
    pat = np.zeros((1, n), np.uint32)
    pat[0, : n // 2] = n // 2 - np.arange(n // 2)   # init_operand (NTT.cu:10-15)
    pat = np.tile(pat, (reps, 1))
    a = _dev(ntt, pat, dev)
    b = torch.empty_like(a)
    ntt.poly_ntt_oop(b, a, ps)
    assert np.array_equal(_u32(ntt, a), pat)
    assert np.array_equal(_u32(ntt, b), oracle.poly_ntt(pat, ps))
    ntt.poly_invntt_oop(a, b, ps)
    assert np.array_equal(_u32(ntt, a), pat)


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_polymul_composition(ntt, oracle, dev, ps):
    """INV(FWD(a) o FWD(b)) through poly_pointwise == the oracle product; the
    all-ones KAT z[k] = 2k + 2 - n mod q (NTT.cu:2360, 2433-2438)."""
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    a = oracle.fill_uniform(5, ps, 1, 0)
    b = oracle.fill_uniform(5, ps, 2, 0)
    a[4] = 1
    b[4] = 1
    ta, tb = _dev(ntt, a, dev), _dev(ntt, b, dev)
    tc = torch.empty_like(ta)
    ntt.poly_ntt(ta, ps)
    ntt.poly_ntt(tb, ps)
    ntt.poly_pointwise(tc, ta, tb, ps)
    ntt.poly_invntt(tc, ps)
    c = _u32(ntt, tc)
    assert np.array_equal(c, oracle.poly_mul(a, b, ps))
    assert np.array_equal(c[4], ((2 * np.arange(n) + 2 - n) % q).astype(np.uint32))


def test_large_nussbaumer_unsupported(ntt, dev):
    """Nussbaumer splits n = 1024 / 2048 only (the reference's routine is
    n = 1024): NTT_ERR_PARAM for the large sets, nothing launched."""
    L = ntt.lib()
    for ps in (3, 4):
        n = ntt.param_info(ps)["n"]
        t = torch.zeros(2 * n, dtype=torch.int32, device=dev)
        u = torch.zeros_like(t)
        p, q = t.data_ptr(), u.data_ptr()
        assert L.poly_mul_nussbaumer(q, p, p, 2, ps, 0, None) == ntt.NTT_ERR_PARAM
        assert L.poly_ntt(p, None, 0, ps, None) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("ps", LARGE_SETS)
@pytest.mark.parametrize("batch", [1, 2, 5, 7, 64, 389, 600])
def test_large_poly_mul_random(ntt, oracle, dev, ps, batch):
    """Fused products, bit-exact against the oracle, over partial and full
    workgroup steps: n = 4096 up to 512 products on the latency kernel
    (ntt_lat.hpp), 600 on k_poly_mul_big (one wave per product, 8 per
    workgroup), n = 8192 on k_poly_mul_large (poly_mul: 4 products per step on
    8-wave workgroups; poly_mul_ntt: 8 on 16-wave ones) -- 5, 7 and 389 are
    multiples of none of them."""
    a = oracle.fill_uniform(batch, ps, 0x3A + batch, 0)
    b = oracle.fill_uniform(batch, ps, 0x3B + batch, 0)
    ta, tb = _dev(ntt, a, dev), _dev(ntt, b, dev)
    tc = torch.empty_like(ta)
    ntt.poly_mul(tc, ta, tb, ps)
    want = oracle.poly_mul(a, b, ps)
    assert np.array_equal(_u32(ntt, tc), want)
    assert np.array_equal(_u32(ntt, ta), a) and np.array_equal(_u32(ntt, tb), b)
    # b-hat = poly_ntt(b): the second operand already in the NTT domain
    tbh = _dev(ntt, b, dev)
    ntt.poly_ntt(tbh, ps)
    tc2 = torch.empty_like(ta)
    ntt.poly_mul_ntt(tc2, ta, tbh, ps)
    assert np.array_equal(_u32(ntt, tc2), want)
    torch.cuda.synchronize()
    assert ntt.sync_expiries() == 0


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_poly_mul_kat_aliasing_lazy(ntt, oracle, dev, ps):
    """All-ones KAT z[k] = 2k + 2 - n mod q (NTT.cu:2360, 2433-2438), the
    init_operand pattern (NTT.cu:10-15), c aliasing a / b / both, inputs in
    [q, 2q) and edge operands."""
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    ones = np.ones((1, n), np.uint32)
    t1 = _dev(ntt, ones, dev)
    tc = torch.empty_like(t1)
    ntt.poly_mul(tc, t1, t1, ps)
    assert np.array_equal(_u32(ntt, tc)[0], ((2 * np.arange(n) + 2 - n) % q).astype(np.uint32))
    pat = np.zeros((1, n), np.uint32)
    pat[0, : n // 2] = n // 2 - np.arange(n // 2)
    tp = _dev(ntt, pat, dev)
    ntt.poly_mul(tc, tp, tp, ps)
    assert np.array_equal(_u32(ntt, tc), oracle.poly_mul(pat, pat, ps))

    a = oracle.fill_uniform(9, ps, 0xA1, 0)
    b = oracle.fill_uniform(9, ps, 0xB1, 0)
    a[0] = 0
    b[1] = q - 1
    a[2] = np.eye(1, n, n - 1, dtype=np.uint32)[0]   # x^(n-1): negacyclic wrap
    b[2] = np.eye(1, n, 1, dtype=np.uint32)[0]
    want = oracle.poly_mul(a, b, ps)
    assert np.array_equal(want[2], ((q - 1) * np.eye(1, n, 0, dtype=np.uint64)[0] % q).astype(np.uint32))
    for alias in ("a", "b"):
        ta, tb = _dev(ntt, a, dev), _dev(ntt, b, dev)
        out = ta if alias == "a" else tb
        ntt.poly_mul(out, ta, tb, ps)
        assert np.array_equal(_u32(ntt, out), want), alias
    ta = _dev(ntt, a, dev)
    ntt.poly_mul(ta, ta, ta, ps)
    assert np.array_equal(_u32(ntt, ta), oracle.poly_mul(a, a, ps))
    al = (a.astype(np.uint64) + q).astype(np.uint32)
    bl = (b.astype(np.uint64) + q).astype(np.uint32)
    ta, tb = _dev(ntt, al, dev), _dev(ntt, bl, dev)
    tc = torch.empty_like(ta)
    ntt.poly_mul(tc, ta, tb, ps)
    assert np.array_equal(_u32(ntt, tc), want)
    # b-hat with entries in [q, 2q) (the forward's lazy range is allowed)
    bh = (oracle.poly_ntt(b, ps).astype(np.uint64) + q).astype(np.uint32)
    tbh = _dev(ntt, bh, dev)
    ta = _dev(ntt, a, dev)
    ntt.poly_mul_ntt(tbh, ta, tbh, ps)
    assert np.array_equal(_u32(ntt, tbh), want)


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_bit_reversed_orders(ntt, oracle, dev, ps):
    """poly_bitrev_copy (bit_reverse_copy_tbl_gpu, NTT.cu:487-492) at
    log2 n = 12 / 13 bits, in and out of place; poly_ntt_bitrev =
    bitrev(poly_ntt); poly_invntt_bitrev on bit-reversed input = the CT
    inverse (oracle_poly_invntt_ct) = poly_invntt."""
    # all on the small-batch kernels; both sides of every switch point of the
    # bit-reversed entry points (the one-launch batch kernels, ntt_big.hpp
    # BR = true, above it) are test_gpu_parity.py::test_latency_switch_boundary's
    for batch in (1, 3, 130, 600):
        x = oracle.fill_uniform(batch, ps, 0xB17 + batch, 0)
        tx = _dev(ntt, x, dev)
        ty = torch.empty_like(tx)
        ntt.poly_bitrev_copy(ty, tx, ps)
        assert np.array_equal(_u32(ntt, ty), oracle.bit_reverse_copy(x, ps))
        ntt.poly_bitrev_copy(ty, ty, ps)   # an involution, in place
        assert np.array_equal(_u32(ntt, ty), x)
        X = oracle.poly_ntt(x, ps)
        ntt.poly_ntt_bitrev(ty, tx, ps)
        assert np.array_equal(_u32(ntt, ty), oracle.bit_reverse_copy(X, ps))
        assert np.array_equal(_u32(ntt, tx), x)
        ntt.poly_ntt_bitrev(tx, tx, ps)
        assert np.array_equal(_u32(ntt, tx), oracle.bit_reverse_copy(X, ps))
        Xb = oracle.bit_reverse_copy(X, ps)
        tX = _dev(ntt, Xb, dev)
        ntt.poly_invntt_bitrev(ty, tX, ps)
        assert np.array_equal(_u32(ntt, ty), x)
        ntt.poly_invntt_bitrev(tX, tX, ps)
        assert np.array_equal(_u32(ntt, tX), x)
        # an arbitrary bit-reversed-order vector vs the oracle's CT inverse
        # (oracle_poly_invntt_ct takes natural order and bit-reverses itself)
        Ybr = oracle.fill_uniform(batch, ps, 0xB18 + batch, 0)
        tY = _dev(ntt, Ybr, dev)
        ntt.poly_invntt_bitrev(tY, tY, ps)
        assert np.array_equal(_u32(ntt, tY), oracle.poly_invntt_ct(oracle.bit_reverse_copy(Ybr, ps), ps))


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_poly_mul_host(ntt, oracle, ps):
    """poly_mul_host through the streamed host context at n = 4096 / 8192
    (ragged last chunk)."""
    a = oracle.fill_uniform(37, ps, 0x40, 0)
    b = oracle.fill_uniform(37, ps, 0x41, 0)
    c = np.empty_like(a)
    with ntt.HostContext(ps, chunk_polys=16, nslots=2) as h:
        h.mul(c, a, b)
    assert np.array_equal(c, oracle.poly_mul(a, b, ps))


@pytest.mark.slow
@pytest.mark.parametrize("ps,batch", [("p-III-4096", 1 << 18), ("p-III-8192", (1 << 17) + 3)])
def test_large_full_batch_properties(ntt, oracle, dev, ps, batch):
    """4-GiB batches: round trip on device, sampled polys vs the oracle, linearity."""
    n, q = ntt.param_info(ps)["n"], ntt.param_info(ps)["q"]
    x = torch.empty(batch * n, dtype=torch.int32, device=dev)
    ntt.fill_uniform(x, ps, 0x5EED0006, 0)
    ref = x.clone()
    ntt.poly_ntt(x, ps)
    rng = np.random.default_rng(2)
    idx = np.unique(np.concatenate([[0, batch - 1], rng.integers(0, batch, 62)]))
    sel = torch.as_tensor(idx, device=dev)
    assert np.array_equal(ntt.to_numpy_u32(x.view(batch, n)[sel]),
                          oracle.poly_ntt(ntt.to_numpy_u32(ref.view(batch, n)[sel]), ps))
    X = x.clone()
    ntt.poly_invntt(x, ps)
    assert torch.equal(x, ref)
    # linearity: NTT(a) + NTT(b) == NTT(a + b mod q) on the whole batch
    b = torch.empty_like(x)
    ntt.fill_uniform(b, ps, 0x5EED0007, 0)
    s = (((ref.to(torch.int64) & 0xFFFFFFFF) + (b.to(torch.int64) & 0xFFFFFFFF)) % q).to(torch.int32)
    del ref, x
    ntt.poly_ntt(b, ps)
    ntt.poly_ntt(s, ps)
    lhs = ((X.to(torch.int64) & 0xFFFFFFFF) + (b.to(torch.int64) & 0xFFFFFFFF)) % q
    assert torch.equal(lhs, s.to(torch.int64) & 0xFFFFFFFF)


@pytest.mark.slow
@pytest.mark.parametrize("ps,batch", [("p-III-4096", (1 << 18) + 5), ("p-III-8192", (1 << 17) + 1)])
def test_large_poly_mul_full_batch_properties(ntt, oracle, dev, ps, batch):
    """3 x 4-GiB operands: sampled products vs the oracle, commutativity over
    the whole batch, poly_mul_ntt(a, NTT(b)) == poly_mul(a, b) on the whole
    batch, no expired slot barrier."""
    n = ntt.param_info(ps)["n"]
    a = torch.empty(batch * n, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    ntt.fill_uniform(a, ps, 0x5EED0011, 0)
    ntt.fill_uniform(b, ps, 0x5EED0012, 0)
    c = torch.empty_like(a)
    ntt.poly_mul(c, a, b, ps)
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([[0, batch - 1], rng.integers(0, batch, 30)]))
    sel = torch.as_tensor(idx, device=dev)
    A = ntt.to_numpy_u32(a.view(batch, n)[sel])
    B = ntt.to_numpy_u32(b.view(batch, n)[sel])
    assert np.array_equal(ntt.to_numpy_u32(c.view(batch, n)[sel]), oracle.poly_mul(A, B, ps))
    d = torch.empty_like(a)
    ntt.poly_mul(d, b, a, ps)
    assert torch.equal(c, d)
    ntt.poly_ntt(b, ps)          # b-hat, in place
    ntt.poly_mul_ntt(d, a, b, ps)
    assert torch.equal(c, d)
    torch.cuda.synchronize()
    assert ntt.sync_expiries() == 0


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_slot_barriers_never_expire(ntt, oracle, dev, ps):
    """The per-polynomial barriers' bounded waits (SlotSync) never run out,
    over partial and full workgroups, in place and out of place."""
    n = ntt.param_info(ps)["n"]
    for batch in (5, 4099):
        x = torch.empty(batch * n, dtype=torch.int32, device=dev)
        ntt.fill_uniform(x, ps, 0x5107 + batch, 0)
        ref = x.clone()
        ntt.poly_ntt(x, ps)
        ntt.poly_invntt(x, ps)
        assert torch.equal(x, ref)
        y = torch.empty_like(x)
        ntt.poly_mul(y, x, x, ps)
        ntt.poly_mul_ntt(y, x, y, ps)
    torch.cuda.synchronize()
    assert ntt.sync_expiries() == 0


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_expired_slot_barrier_writes_sentinel(ntt, dev, ps):
    """An expired slot-barrier wait (the n = 8192 fused products'
    multi-wave kernels, ntt_large.hpp) fails loudly: in the test build whose
    waits always expire (lib/libqtesla_ntt_syncfail.so, LARGE_SLOT_SYNC_SPIN=0,
    the same sources), every stored coefficient is the non-canonical sentinel
    0xFFFFFFFF (>= q, caught by any range check without a device sync) and
    the device counter behind ntt_sync_expiries() counts the expiries."""
    import ctypes
    import os
    path = os.path.join(os.path.dirname(ntt.LIB_PATH), "libqtesla_ntt_syncfail.so")
    if not os.path.exists(path):   # a tree built with plain `make all`: build the test library
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(path)), "testlibs"], check=False)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: build with `make -C ntt-gpu-qtesla_amd testlibs`")
    ntt.lib()   # the HIP runtime torch loaded is bound first
    L = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.poly_ntt.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    L.poly_invntt.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    L.poly_mul.argtypes = [vp, vp, vp, sz, ctypes.c_int, vp]
    L.ntt_sync_expiries.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
    psn = ntt.PARAM_SETS[ps]
    n = ntt.param_info(ps)["n"]
    # the transforms run one wave per polynomial (ntt_big.hpp): no slot
    # barrier, so the always-expiring build transforms exactly
    for fn, ref in ((L.poly_ntt, ntt.poly_ntt), (L.poly_invntt, ntt.poly_invntt)):
        x = torch.empty(37 * n, dtype=torch.int32, device=dev)
        ntt.fill_uniform(x, ps, 0x5E17, 0)
        want = ref(x.clone(), ps)
        torch.cuda.synchronize()
        assert fn(x.data_ptr(), None, 37, psn, None) == 0
        torch.cuda.synchronize()
        assert torch.equal(x, want)
    x = torch.empty(37 * n, dtype=torch.int32, device=dev)
    ntt.fill_uniform(x, ps, 0x5E18, 0)
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    assert L.poly_mul(y.data_ptr(), x.data_ptr(), x.data_ptr(), 37, psn, None) == 0
    torch.cuda.synchronize()
    c = ctypes.c_uint32(0)
    assert L.ntt_sync_expiries(ctypes.byref(c)) == 0
    if n == 4096:
        # n = 4096 products also run one wave per polynomial (k_poly_mul_big)
        want = torch.empty_like(x)
        ntt.poly_mul(want, x, x, ps)
        torch.cuda.synchronize()
        assert torch.equal(y, want)
        assert c.value == 0
    else:
        assert bool((y == -1).all()), "the fused product fails loudly too"
        assert c.value > 0
    assert ntt.sync_expiries() == 0   # the product library's own counter is untouched


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_host_driver_kat(ps):
    """The C++ host driver (reference CLI) at n = 4096 / 8192: CT-GS
    composition and fused product report the all-ones KAT as Identical, the
    transform round trip and the host pipeline pass; Nussbaumer (option 11)
    fails with the library's NTT_ERR_PARAM."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ntt-gpu-qtesla_amd", "bin", "ntt_main")
    for opt, batch in (("6", "4"), ("7", "4"), ("9", "300"), ("10", "1500")):
        args = [exe, "-speedgpu", opt, "-param", ps, "-batch", batch] + (["-r", "5"] if opt == "9" else [])
        r = subprocess.run(args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "Identical." in r.stdout, r.stdout + r.stderr
    r = subprocess.run([exe, "-speedgpu", "11", "-param", ps, "-batch", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
