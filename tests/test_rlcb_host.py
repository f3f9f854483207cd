"""Batch-wide RLC check with the Pippenger MSM (charon_amd/csrc/rlcb.h) on the host build of the kernel stages:

* the MSM (counting sort by 16-bit digit, bucket sums, segment folds, window combination) equals the naive
  sum_i [k_i] P_i from the oracle, including zero scalars, repeated points (doublings inside a bucket) and digits
  at the window edges;
* an honest batch passes the batch-wide check itself (the window stages then have nothing left to decide);
* a batch with invalid items fails it, and the window/fallback stages give exactly per-item Verify, including
  the cancellation case that only the random scalars catch.
"""
import ctypes
import random

from oracle import bls12381 as bls
from tests.hostlib import buf, lib
from tests.rlc_cases import fixture_batch, message_table, validator_batch
from tests.test_rlc_host import host_pk, host_sign

SEED = bytes(range(32))


def _aff_bytes(pt):
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(48, "big") for v in (x0, x1, y0, y1))


def test_msm_matches_naive_sum():
    L = lib()
    rng = random.Random(5)
    base = [bls.hash_to_g2(bytes([k]) * 7) for k in range(6)]
    pts = [base[k % 6] for k in range(14)]  # repeats: several points share a bucket
    scal = [rng.randrange(1 << 32) for _ in pts]
    scal[0] = 0                      # skipped
    scal[1] = 1                      # bucket 1 of window 0 only
    scal[2] = 0xFFFF0000             # window 1 only, top bucket
    scal[3] = 0x0001FFFF             # both windows, top bucket of window 0
    scal[4] = scal[5]                # identical (point, scalar) pairs: doubling inside a bucket
    pts[4] = pts[5]
    out = buf(96)
    L.ht_msm_g2(b"".join(_aff_bytes(p) for p in pts), (ctypes.c_uint32 * len(pts))(*scal), len(pts), out)
    want = None
    for p, k in zip(pts, scal):
        want = bls.g2_add(want, bls.g2_mul(p, k))
    assert out.raw == bls.g2_compress(want)


def test_msm_buckets_cut_by_run_lanes():
    """Buckets of ~90 entries over run lanes of MSM_RUN = 64 list entries (rlcb.h msm_run_lane / msm_fix_lane): buckets
    that start a run lane's range, end inside the next one, span three lanes, and whole buckets inside one range."""
    L = lib()
    rng = random.Random(11)
    base = [bls.hash_to_g2(bytes([k]) * 5) for k in range(5)]
    kset = [0x00030002, 0x00030005, 0x0007FFFF]  # shared digits: large buckets in both windows
    pts, scal = [], []
    for i in range(300):
        pts.append(base[i % 5])
        scal.append(kset[rng.randrange(3)] if i % 9 else rng.randrange(1 << 32))
    out = buf(96)
    L.ht_msm_g2(b"".join(_aff_bytes(p) for p in pts), (ctypes.c_uint32 * len(pts))(*scal), len(pts), out)
    mult = {}
    for i, k in enumerate(scal):
        mult[(i % 5, k)] = mult.get((i % 5, k), 0) + 1
    want = None
    for (b, k), c in mult.items():
        want = bls.g2_add(want, bls.g2_mul(base[b], k * c % bls.R))
    assert out.raw == bls.g2_compress(want)


def rlcb(L, pks, msgs, sigs, seed=SEED, counts=None):
    table, idx = message_table(msgs)
    n = len(pks)
    offs = (ctypes.c_uint64 * (len(table) + 1))()
    acc = 0
    for m, t in enumerate(table):
        offs[m] = acc
        acc += len(t)
    offs[len(table)] = acc
    st = (ctypes.c_int32 * max(n, 1))()
    passed = ctypes.c_int32(-1)
    arr = (ctypes.c_uint32 * max(n, 1))(*idx)
    rc = L.ht_rlcb_verify(b"".join(pks), b"".join(sigs), arr, ctypes.c_uint64(n), b"".join(table), offs,
                          ctypes.c_uint64(len(table)), seed, st, ctypes.byref(passed), counts)
    assert rc == 0
    return [st[i] for i in range(n)], passed.value


def test_rlcb_honest_batch_passes_batch_check():
    L = lib()
    pks, msgs, sigs, want = validator_batch(host_sign(L), host_pk(L), 9, 4, seed=21)  # 36 items, 3 chunks
    got, passed = rlcb(L, pks, msgs, sigs)
    assert got == want == [0] * 36
    assert passed == 1


def test_rlcb_invalid_items_fall_back_to_windows():
    L = lib()
    pks, msgs, sigs, want = validator_batch(host_sign(L), host_pk(L), 6, 4, seed=22, bad=(2, 13, 19))
    got, passed = rlcb(L, pks, msgs, sigs)
    assert passed == 0
    for g, w in zip(got, want):
        assert g == w if w is not None else g in (2, 3)


def test_rlcb_cancellation_is_caught():
    """Two partials under one root with their signatures swapped: the unrandomized sums would cancel."""
    L = lib()
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 4, 4, seed=23)
    sigs[5], sigs[6] = sigs[6], sigs[5]
    got, passed = rlcb(L, pks, msgs, sigs)
    assert passed == 0
    assert got == [0] * 5 + [3, 3] + [0] * 9


def test_rlcb_fixture_statuses():
    """Edge encodings: bad keys/signatures and infinity get their final status in stage 1; the rest decide."""
    L = lib()
    pks, msgs, sigs, want = fixture_batch()
    got, _ = rlcb(L, pks, msgs, sigs)
    assert got == want


def test_chunk_count_leaves_a_simd_free():
    """rlcb.h rlcb_chunk_count: ceil(n / 16) chunks unless they fill whole rounds of waves exactly, then one wave
    fewer (at most 18 items per lane); the bench's 1M items on 1,024 wave slots get 65,472 chunks."""
    L = lib()
    f = L.ht_rlcb_chunk_count
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    assert f(1 << 20, 1024) == 65472            # 1,024 waves -> 1,023
    assert f(1 << 20, 0) == 65536               # no device information: plain ceil(n / 16)
    assert f((1 << 20) - 16, 1024) == 65472     # 65,535 chunks: still 1,024 waves, every SIMD -> one wave fewer
    assert f(16 * 64 * 1000, 1024) == 64000     # 1,000 waves: a SIMD is free already
    assert f(16 * 64 * 2048, 1024) == 64 * 2047  # two whole rounds -> one wave fewer
    assert f(100, 1) == 7                       # one wave: never reduced
    assert f(16 * 64 * 9, 9) == 16 * 64 * 9 // 18  # 9 waves -> 8, 18 items per lane (the cap)
    assert f(16 * 64 * 8, 8) == 16 * 64 * 8 // 16  # 8 waves -> 7 would need > 18 per lane: kept


def test_rlcb_uneven_chunks_same_verdicts():
    """Chunks of 17 and 18 items (a chunk count that does not divide the batch, as rlcb_chunk_count makes on the
    device) give the same verdicts: the honest batch passes, the cancellation case fails and falls back exactly."""
    L = lib()
    L.ht_rlcb_set_chunks(ctypes.c_uint64(4))
    try:
        pks, msgs, sigs, want = validator_batch(host_sign(L), host_pk(L), 14, 5, seed=24)  # 70 items
        got, passed = rlcb(L, pks, msgs, sigs)
        assert got == want == [0] * 70 and passed == 1
        sigs[5], sigs[6] = sigs[6], sigs[5]  # same root, swapped: only the scalars catch it
        got, passed = rlcb(L, pks, msgs, sigs)
        assert passed == 0 and got == [0] * 5 + [3, 3] + [0] * 63
    finally:
        L.ht_rlcb_set_chunks(ctypes.c_uint64(0))


def committee_batch(L, sizes, seed, shuffle=False):
    """Committee roots: sizes[m] partials (distinct keys) all signing root m; items grouped by root unless shuffled."""
    rng = random.Random(seed)
    sign, to_pk = host_sign(L), host_pk(L)
    roots = [rng.randbytes(32) for _ in sizes]
    items = [(m, rng.randrange(1, bls.R).to_bytes(32, "big")) for m, k in enumerate(sizes) for _ in range(k)]
    if shuffle:
        rng.shuffle(items)
    pks = [to_pk(sk) for _, sk in items]
    msgs = [roots[m] for m, _ in items]
    sigs = [sign(sk, roots[m]) for m, sk in items]
    return pks, msgs, sigs


def _with_g1_min(L, k, fn):
    L.ht_rlcb_set_g1_min.restype = ctypes.c_uint32
    old = L.ht_rlcb_set_g1_min(ctypes.c_uint32(k))
    try:
        return fn()
    finally:
        L.ht_rlcb_set_g1_min(ctypes.c_uint32(old))


def test_rlcb_g1_msm_committee_roots():
    """g1msm.h: roots with >= min items get one bucket-method sum of [r_i] pk_i and one Miller loop (roots 0 and 1
    here), the small root keeps the per-item path; the batch passes with and without it, items in any order."""
    L = lib()
    for shuffle in (False, True):
        pks, msgs, sigs = committee_batch(L, [40, 24, 3], seed=31, shuffle=shuffle)
        got, passed = _with_g1_min(L, 16, lambda: rlcb(L, pks, msgs, sigs))
        assert got == [0] * 67 and passed == 1
        got, passed = _with_g1_min(L, 0, lambda: rlcb(L, pks, msgs, sigs))
        assert got == [0] * 67 and passed == 1
    # the path is taken: stage 1 skips the 64 large-root items' Shamir multiplications (~600 products each), the
    # chunks pair only the small root
    on, off = (ctypes.c_uint64 * 6)(), (ctypes.c_uint64 * 6)()
    _with_g1_min(L, 16, lambda: rlcb(L, pks, msgs, sigs, counts=on))
    _with_g1_min(L, 0, lambda: rlcb(L, pks, msgs, sigs, counts=off))
    assert off[0] - on[0] > 64 * 500 and on[3] < off[3]


def test_rlcb_g1_msm_failures_fall_back_exactly():
    """Invalid partials inside large roots: a swapped pair (only the scalars catch it), a wrong key, a flipped
    signature bit (final status in stage 1, zero scalars in its slot).  The batch check fails, the windows take
    [r_i] pk_i from the slots (rlcb_mark_lane) and decide each item exactly as with the G1 MSM off."""
    L = lib()
    pks, msgs, sigs = committee_batch(L, [40, 24, 3], seed=32)
    sigs[5], sigs[6] = sigs[6], sigs[5]
    pks[45] = pks[46]
    b = bytearray(sigs[50])
    b[40] ^= 0x04
    sigs[50] = bytes(b)
    got, passed = _with_g1_min(L, 16, lambda: rlcb(L, pks, msgs, sigs))
    ref, ref_passed = _with_g1_min(L, 0, lambda: rlcb(L, pks, msgs, sigs))
    assert passed == ref_passed == 0
    assert got == ref
    assert got[5] == got[6] == got[45] == 3 and got[50] in (2, 3)
    assert [g for i, g in enumerate(got) if i not in (5, 6, 45, 50)] == [0] * 63
