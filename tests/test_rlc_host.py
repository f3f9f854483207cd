"""RLC BatchVerify on the host build of the kernel stages (charon_amd/csrc/rlc.h via tests/native):
statuses must equal per-item tbls.Verify, and honest windows must pass the batched check itself
(not only through the per-item fallback, which would hide a broken combination)."""
import ctypes

from oracle import bls12381 as bls
from tests.hostlib import buf, lib
from tests.rlc_cases import fixture_batch, message_table, validator_batch

SEED = bytes(range(32))


def rlc(L, pks, msgs, sigs, seed=SEED):
    table, idx = message_table(msgs)
    n = len(pks)
    offs = (ctypes.c_uint64 * (len(table) + 1))()
    acc = 0
    for m, t in enumerate(table):
        offs[m] = acc
        acc += len(t)
    offs[len(table)] = acc
    st = (ctypes.c_int32 * max(n, 1))()
    stats = (ctypes.c_uint64 * 3)()
    arr = (ctypes.c_uint32 * max(n, 1))(*idx)
    rc = L.ht_rlc_verify(b"".join(pks), b"".join(sigs), arr, ctypes.c_uint64(n), b"".join(table), offs,
                         ctypes.c_uint64(len(table)), seed, st, stats, None)
    assert rc == 0
    return [st[i] for i in range(n)], list(stats)


def host_sign(L):
    def sign(sk, m):
        out = buf(96)
        assert L.ht_sign(sk, m, len(m), out) == 0
        return out.raw
    return sign


def host_pk(L):
    def pk(sk):
        out = buf(48)
        assert L.ht_sk_to_pk(sk, out) == 0
        return out.raw
    return pk


def test_rlc_fixtures_match_oracle():
    L = lib()
    pks, msgs, sigs, want = fixture_batch()
    got, _ = rlc(L, pks, msgs, sigs)
    assert got == want


def test_rlc_honest_windows_pass_without_fallback():
    L = lib()
    pks, msgs, sigs, want = validator_batch(host_sign(L), host_pk(L), 5, 4, seed=7)  # 20 items: 3 windows
    got, (windows, failed, fallback) = rlc(L, pks, msgs, sigs)
    assert got == want == [0] * 20
    assert windows == 3 and failed == 0 and fallback == 0


def test_rlc_bad_item_fails_only_its_window():
    L = lib()
    bad = (5, 17, 18)
    pks, msgs, sigs, want = validator_batch(host_sign(L), host_pk(L), 6, 4, seed=9, bad=bad)  # 24 items
    got, (windows, failed, fallback) = rlc(L, pks, msgs, sigs)
    for i, (g, w) in enumerate(zip(got, want)):
        if w is None:
            assert g in (2, 3), i
        else:
            assert g == w, i
    # oracle agrees on every item
    assert got == [bls.verify_status(p, m, s) for p, m, s in zip(pks, msgs, sigs)]
    # item 18's flipped bit may fail decoding (status 2: excluded before batching) -> its window may pass
    assert windows == 3 and 1 <= failed <= 2


def test_rlc_seed_independent():
    L = lib()
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 2, 4, seed=11, bad=(3,))
    a, _ = rlc(L, pks, msgs, sigs, seed=bytes(32))
    b, _ = rlc(L, pks, msgs, sigs, seed=b"\xff" * 32)
    assert a == b


def rlc_keys(L, table_pks, key_idx, msgs, sigs, seed=SEED):
    table, idx = message_table(msgs)
    n = len(sigs)
    offs = (ctypes.c_uint64 * (len(table) + 1))()
    acc = 0
    for m, t in enumerate(table):
        offs[m] = acc
        acc += len(t)
    offs[len(table)] = acc
    st = (ctypes.c_int32 * max(n, 1))()
    tst = (ctypes.c_int32 * max(len(table_pks), 1))()
    stats = (ctypes.c_uint64 * 3)()
    rc = L.ht_rlc_verify_keys(b"".join(table_pks), ctypes.c_uint64(len(table_pks)),
                              (ctypes.c_uint32 * max(n, 1))(*key_idx), b"".join(sigs),
                              (ctypes.c_uint32 * max(n, 1))(*idx), ctypes.c_uint64(n), b"".join(table), offs,
                              ctypes.c_uint64(len(table)), seed, st, tst, stats)
    assert rc == 0
    return [st[i] for i in range(n)], [tst[i] for i in range(len(table_pks))], list(stats)


def test_pubshare_table_verify_matches_wire_verify():
    """k_verify_keys body: key from the decoded table == op_verify on the wire key (fixtures)."""
    L = lib()
    pks, msgs, sigs, want = fixture_batch()
    got = [L.ht_verify_key(p, m, len(m), s) for p, m, s in zip(pks, msgs, sigs)]
    assert got == want


def test_rlc_with_pubshare_table():
    """Keys by table index (shuffled table, repeated keys, one bad table entry) == per-item Verify."""
    L = lib()
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 4, 4, seed=17, bad=(6,))
    order = list(range(len(pks)))[::-1]
    table_pks = [pks[i] for i in order] + [bytes(48)]       # last entry: not a valid encoding
    key_idx = [len(pks) - 1 - i for i in range(len(pks))]
    key_idx[11] = len(pks)                                   # item 11 names the bad key
    got, tst, (windows, failed, fallback) = rlc_keys(L, table_pks, key_idx, msgs, sigs)
    assert tst == [0] * len(pks) + [1]
    wire = [bls.verify_status(table_pks[k], m, s) for k, m, s in zip(key_idx, msgs, sigs)]
    assert got == wire
    assert got[11] == 1 and got[6] == 3 and got.count(0) == 14
    assert windows == 2 and failed == 1
