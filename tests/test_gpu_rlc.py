"""GPU parity of RLC BatchVerify (hipbls_batch_verify_rlc) through the C-ABI: per-item statuses
identical to individual tbls.Verify (hipbls_verify_batch, itself pinned to the oracle and herumi
KATs), on the oracle fixtures, on validator-shaped batches with corruptions, and at a C4-shaped size
through the size-independent property "honest windows pass the batched check, corrupted items and
only they fail"."""
import random

import pytest

from tests.rlc_cases import fixture_batch, validator_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def sign_batch_fns(impl):
    cache = {}

    def pk(sk):
        if sk not in cache:
            cache[sk] = impl.secret_to_public_key(sk)
        return cache[sk]
    return impl.sign, pk


def test_rlc_fixtures_match_oracle(impl):
    pks, msgs, sigs, want = fixture_batch()
    assert impl.batch_verify_rlc_status(pks, msgs, sigs, seed=bytes(32)) == want


def test_rlc_empty(impl):
    assert impl.batch_verify_rlc_status([], [], []) == []


def test_rlc_honest_no_fallback(impl):
    sign, pk = sign_batch_fns(impl)
    pks, msgs, sigs, _ = validator_batch(sign, pk, 16, 4, seed=3)
    assert impl.batch_verify_rlc_status(pks, msgs, sigs) == [0] * 64
    assert impl.rlc_stats() == (8, 0, 0)


def test_rlc_matches_individual_with_corruptions(impl):
    sign, pk = sign_batch_fns(impl)
    pks, msgs, sigs, want = validator_batch(sign, pk, 32, 4, seed=5, bad=(0, 9, 10, 63, 64, 127))
    got = impl.batch_verify_rlc_status(pks, msgs, sigs)
    assert got == impl.batch_verify_status(pks, msgs, sigs)
    for g, w in zip(got, want):
        assert g == w if w is not None else g in (2, 3)


def test_rlc_distinct_and_shared_messages(impl):
    """Every item its own message (C2 shape) and one message for all (committee-shared root)."""
    rng = random.Random(12)
    sks = [rng.randrange(1, 2 ** 254).to_bytes(32, "big") for _ in range(40)]
    pks, _ = impl.secret_to_public_key_batch(sks)
    distinct = [rng.randbytes(32) for _ in range(40)]
    sigs, _ = impl.sign_batch(sks, distinct)
    assert impl.batch_verify_rlc_status(pks, distinct, sigs) == [0] * 40
    assert impl.rlc_stats()[1] == 0
    shared = [b"committee root".ljust(32, b"\0")] * 40
    sigs2, _ = impl.sign_batch(sks, shared)
    sigs2[17] = sigs[17]  # signature over another root
    got = impl.batch_verify_rlc_status(pks, shared, sigs2)
    assert got == [0] * 17 + [3] + [0] * 22
    assert impl.rlc_stats() == (5, 1, 8)


def test_rlc_non_adjacent_messages(impl):
    """Interleaved messages (no grouping by the caller) stay correct, only costlier."""
    rng = random.Random(13)
    sks = [rng.randrange(1, 2 ** 254).to_bytes(32, "big") for _ in range(24)]
    pks, _ = impl.secret_to_public_key_batch(sks)
    roots = [rng.randbytes(32) for _ in range(3)]
    msgs = [roots[i % 3] for i in range(24)]
    sigs, _ = impl.sign_batch(sks, msgs)
    assert impl.batch_verify_rlc_status(pks, msgs, sigs) == [0] * 24
    assert impl.rlc_stats()[1] == 0


def test_rlc_large_properties(impl):
    """C4 shape at reduced count (4 partials per validator, one root each, 0.5% corrupted)."""
    rng = random.Random(21)
    n_dv, t = 2048, 4
    n = n_dv * t
    sks = [rng.randrange(1, 2 ** 254).to_bytes(32, "big") for _ in range(256)]
    keys, _ = impl.secret_to_public_key_batch(sks)
    roots = [rng.randbytes(32) for _ in range(n_dv)]
    owner = [rng.randrange(256) for _ in range(n)]
    msgs = [roots[i // t] for i in range(n)]
    sigs, st = impl.sign_batch([sks[o] for o in owner], msgs)
    assert set(st) == {0}
    pks = [keys[o] for o in owner]
    bad = sorted(rng.sample(range(n), n // 200))
    for i in bad:
        pks[i] = keys[(owner[i] + 1) % 256]
    got = impl.batch_verify_rlc_status(pks, msgs, sigs)
    assert [i for i, s in enumerate(got) if s != 0] == bad
    assert all(got[i] == 3 for i in bad)
    windows, failed, fallback = impl.rlc_stats()
    assert windows == n // 8
    assert failed == len({i // 8 for i in bad})
    assert fallback == 8 * failed


# ---------------------------------------------------------------- resident pubshare table (§8f.2)
def test_pubshare_table_verify_and_rlc_match_wire(impl):
    """Keys by table index give exactly the wire-format statuses (Verify and RLC), including a bad
    table entry, an infinity key and an index outside the table (argument error)."""
    from tests.rlc_cases import fixture_batch
    pks, msgs, sigs, want = fixture_batch()
    table = list(dict.fromkeys(pks))  # distinct keys, first-seen order
    tst = impl.load_pubshares(table)
    assert tst == [1 if impl.batch_verify_status([k], [b"x"], [sigs[0]])[0] == 1 else 0 for k in table]
    kidx = [table.index(p) for p in pks]
    assert impl.batch_verify_keys_status(kidx, msgs, sigs) == want
    assert impl.batch_verify_rlc_keys_status(kidx, msgs, sigs) == want
    with pytest.raises(ValueError):
        impl.batch_verify_keys_status([len(table)], [msgs[0]], [sigs[0]])


def test_pubshare_table_large(impl):
    sign, pk = sign_batch_fns(impl)
    pks, msgs, sigs, _ = validator_batch(sign, pk, 64, 4, seed=31, bad=(3, 100, 200))
    table = sorted(set(pks))
    assert set(impl.load_pubshares(table)) == {0}
    kidx = [table.index(p) for p in pks]
    wire = impl.batch_verify_status(pks, msgs, sigs)
    assert impl.batch_verify_keys_status(kidx, msgs, sigs) == wire
    assert impl.batch_verify_rlc_keys_status(kidx, msgs, sigs) == wire
    assert impl.batch_verify_rlc_status(pks, msgs, sigs) == wire
