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


def rlcb(L, pks, msgs, sigs, seed=SEED):
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
                          ctypes.c_uint64(len(table)), seed, st, ctypes.byref(passed), None)
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
