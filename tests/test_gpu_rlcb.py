"""Batch-wide RLC check with the Pippenger MSM (charon_amd/csrc/rlcb.h) on the GPU, through the C-ABI.

Statuses must equal per-item Verify in every mode (hipbls_rlc_set_mode), and the batch-wide verdict itself is
checked through hipbls_rlc_batch_stats: an all-valid batch must pass it (a broken MSM, chunk product or final
exponentiation would fail it and hide behind the window fallback), a batch with an invalid item must fail it,
including the swapped-signature case that only the random scalars catch.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import RLC_AUTO, HipBLS
    b = HipBLS()
    yield b
    b.set_rlc_mode(RLC_AUTO)


@pytest.fixture(scope="module")
def keys(impl):
    rng = random.Random(77)
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(256)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) == {0}
    return sks, pks


def _batch(impl, keys, n_val, per_val, seed, n_roots=0):
    """n_val validators x per_val partials, grouped by validator; one root each, or n_roots committee roots."""
    sks, pks = keys
    rng = random.Random(seed)
    roots = [rng.randbytes(32) for _ in range(n_roots or n_val)]
    idx, M = [], []
    for v in range(n_val):
        r = roots[v * len(roots) // n_val]
        for _ in range(per_val):
            idx.append(rng.randrange(len(sks)))
            M.append(r)
    S, st = impl.sign_batch([sks[k] for k in idx], M)
    assert set(st) == {0}
    return idx, [pks[k] for k in idx], M, S


def _run(impl, mode, P, M, S, seed=bytes(range(32))):
    impl.set_rlc_mode(mode)
    a0, p0, _ = impl.rlc_batch_stats()
    got = impl.batch_verify_rlc_status(P, M, S, seed=seed)
    a1, p1, last = impl.rlc_batch_stats()
    return got, a1 - a0, p1 - p0, last


@pytest.mark.parametrize("n_val,per_val,n_roots", [(1, 1, 0), (5, 3, 0), (17, 1, 0), (300, 4, 0), (256, 8, 3),
                                                   (1024, 4, 0), (2048, 4, 16)])
def test_honest_batch_passes_batch_check(impl, keys, n_val, per_val, n_roots):
    from charon_amd.tbls import RLC_BATCH
    _, P, M, S = _batch(impl, keys, n_val, per_val, n_val * 31 + per_val, n_roots)
    got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
    assert got == [0] * len(P)
    assert (att, passed, last) == (1, 1, 1)


def test_invalid_items_fail_batch_check_and_windows_decide(impl, keys):
    from charon_amd.tbls import RLC_BATCH, RLC_WINDOWS
    sks, pks = keys
    idx, P, M, S = _batch(impl, keys, 500, 4, 5)
    bad = [3, 777, 1999]
    wrong, _ = impl.sign_batch([sks[(idx[i] + 1) % len(sks)] for i in bad], [M[i] for i in bad])
    for i, w in zip(bad, wrong):
        S[i] = w
    flip = bytearray(S[1000])
    flip[40] ^= 0x04
    S[1000] = bytes(flip)
    want = impl.batch_verify_status(P, M, S)
    assert sum(1 for w in want if w != 0) == 4
    got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
    assert (att, passed, last) == (1, 0, 0)
    assert got == want
    got_w, att_w, _, _ = _run(impl, RLC_WINDOWS, P, M, S)
    assert att_w == 0 and got_w == want


def test_swapped_signatures_fail_batch_check(impl, keys):
    """Two partials under one root with their signatures swapped: an unrandomized sum would cancel."""
    from charon_amd.tbls import RLC_BATCH
    _, P, M, S = _batch(impl, keys, 256, 4, 6)
    S[9], S[10] = S[10], S[9]
    got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
    assert (att, passed, last) == (1, 0, 0)
    assert got == [0] * 9 + [3, 3] + [0] * (len(P) - 11)


def test_fixture_edges_in_batch_mode(impl):
    from charon_amd.tbls import RLC_BATCH
    from tests.rlc_cases import fixture_batch
    P, M, S, want = fixture_batch()
    got, att, _, _ = _run(impl, RLC_BATCH, P, M, S)
    assert att == 1 and got == want


def test_key_table_batch_check(impl, keys):
    from charon_amd.tbls import RLC_BATCH
    sks, pks = keys
    assert set(impl.load_pubshares(pks)) == {0}
    idx, P, M, S = _batch(impl, keys, 400, 4, 7)
    impl.set_rlc_mode(RLC_BATCH)
    a0, p0, _ = impl.rlc_batch_stats()
    got = impl.batch_verify_rlc_keys_status(idx, M, S, seed=bytes(32))
    a1, p1, last = impl.rlc_batch_stats()
    assert got == [0] * len(idx)
    assert (a1 - a0, p1 - p0, last) == (1, 1, 1)


def test_auto_policy_backs_off_after_a_failure(impl, keys):
    """AUTO: small batches stay on windows; after a failed batch-wide check the next 8 large calls run windows only,
    then the batch-wide check is tried again."""
    from charon_amd.tbls import RLC_AUTO
    sks, _ = keys
    _, Ps, Ms, Ss = _batch(impl, keys, 100, 4, 8)  # 400 items < 1,024
    got, att, _, _ = _run(impl, RLC_AUTO, Ps, Ms, Ss)
    assert att == 0 and got == [0] * 400
    idx, P, M, S = _batch(impl, keys, 300, 4, 9)  # 1,200 items
    good = list(S)
    wrong, _ = impl.sign_batch([sks[(idx[5] + 1) % len(sks)]], [M[5]])
    S[5] = wrong[0]
    got, att, _, last = _run(impl, RLC_AUTO, P, M, S)
    assert att == 1 and last == 0 and got[5] == 3 and got.count(0) == len(P) - 1
    for _ in range(8):
        got, att, _, _ = _run(impl, RLC_AUTO, P, M, good)
        assert att == 0 and got == [0] * len(P)
    got, att, passed, last = _run(impl, RLC_AUTO, P, M, good)
    assert (att, passed, last) == (1, 1, 1) and got == [0] * len(P)


def test_verdict_ring_wraps(impl, keys):
    """More batch checks than verdict slots (8): every verdict is read back once, the newest one is `last`."""
    from charon_amd.tbls import RLC_BATCH
    sks, _ = keys
    idx, P, M, S = _batch(impl, keys, 64, 4, 10)
    impl.set_rlc_mode(RLC_BATCH)
    a0, p0, _ = impl.rlc_batch_stats()
    for _ in range(11):
        assert impl.batch_verify_rlc_status(P, M, S, seed=bytes(32)) == [0] * len(P)
    wrong, _ = impl.sign_batch([sks[(idx[0] + 1) % len(sks)]], [M[0]])
    bad = [wrong[0]] + S[1:]
    got = impl.batch_verify_rlc_status(P, M, bad, seed=bytes(32))
    a1, p1, last = impl.rlc_batch_stats()
    assert got[0] == 3 and got[1:] == [0] * (len(P) - 1)
    assert (a1 - a0, p1 - p0, last) == (12, 11, 0)


def test_g1_msm_edges(impl, keys):
    """The G1 MSM per committee root (g1msm.h) at its edges, against per-item Verify and the batch verdict:
    a large root whose every item fails to decode (zero scalars: an empty sum, Miller value 1), the G1 path taken
    with no root large enough (40 roots x 12 items: the kernels run with nl = 0), every root large (threshold 1),
    and the resident key table with committee roots (keys from the table into the slots)."""
    from charon_amd.tbls import RLC_BATCH
    sks, pks = keys
    # (a) root 0's 80 items all broken, root 1's 80 honest
    idx, P, M, S = _batch(impl, keys, 40, 4, 41, n_roots=2)
    for i in range(80):
        b = bytearray(S[i])
        b[0] &= 0x7F  # compression flag cleared: ERR_SIGNATURE in stage 1
        S[i] = bytes(b)
    want = impl.batch_verify_status(P, M, S)
    assert want == [2] * 80 + [0] * 80
    got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
    assert got == want and (att, passed, last) == (1, 1, 1)
    # (b) G1 path on, no large root
    _, P, M, S = _batch(impl, keys, 120, 4, 42, n_roots=40)
    got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
    assert got == [0] * 480 and (att, passed, last) == (1, 1, 1)
    # (c) every root large; one swapped pair inside a root still caught
    old = impl.set_rlc_g1_msm_min(1)
    try:
        _, P, M, S = _batch(impl, keys, 128, 4, 43, n_roots=8)
        got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
        assert got == [0] * 512 and (att, passed, last) == (1, 1, 1)
        S[20], S[21] = S[21], S[20]
        got, att, passed, last = _run(impl, RLC_BATCH, P, M, S)
        assert (att, passed, last) == (1, 0, 0) and got == [0] * 20 + [3, 3] + [0] * 490
    finally:
        impl.set_rlc_g1_msm_min(old)
    # (d) resident key table, committee roots
    assert set(impl.load_pubshares(pks)) == {0}
    idx, P, M, S = _batch(impl, keys, 512, 4, 44, n_roots=4)
    impl.set_rlc_mode(RLC_BATCH)
    a0, p0, _ = impl.rlc_batch_stats()
    got = impl.batch_verify_rlc_keys_status(idx, M, S, seed=bytes(32))
    a1, p1, last = impl.rlc_batch_stats()
    assert got == [0] * len(idx) and (a1 - a0, p1 - p0, last) == (1, 1, 1)
