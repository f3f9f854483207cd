"""Points of small order through every device layout (VERDICT r02 "Next round" 1, ADVICE r02 lg2.h / kernels.h).

Verify takes the signature's G2 membership from its own Miller loop (charon_amd/csrc/pairing.h
g2_subgroup_from_miller; the lane-pair kernel on its odd lane, kernels.h k_verify_pair_lg2).  A signature of order
13 or 23 makes a doubling or addition step of that loop exceptional (Z = 0); herumi rejects it at deserialization
(/root/reference/tbls/herumi.go:291-294), status 2, whatever the key or message.  Public keys with G1 cofactor
torsion (orders 3 and 11) go through the phi subgroup test (herumi.go:286-289, status 1).

The cases and their statuses come from the oracle (tests/golden/make_fixtures.py `small_order_cases`); each one is
sent through: one lane per check, a lane pair per check, the automatic choice, the submission queue, the key table,
RLC windows (window + fallback), the batch-wide RLC check, FastAggregateVerify, ThresholdAggregate (plain and fused
with the aggregate Verify) and eth2util/signing.Verify.
"""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def h(s):
    return bytes.fromhex(s)


@pytest.fixture(scope="module")
def so():
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        return json.load(f)["small_order"]


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def _cases(so):
    c = so["verify"]
    return [h(x["pk"]) for x in c], [h(x["msg"]) for x in c], [h(x["sig"]) for x in c], [x["status"] for x in c]


def _padded(impl, so, n_honest, seed):
    """The small-order cases spread through a batch of honest items (so RLC windows mix them with valid partials)."""
    pks, msgs, sigs, want = _cases(so)
    rng = random.Random(seed)
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(16)]
    hpk, _ = impl.secret_to_public_key_batch(sks)
    roots = [rng.randbytes(32) for _ in range(n_honest // 4 + 1)]
    owner = [rng.randrange(16) for _ in range(n_honest)]
    hm = [roots[i // 4] for i in range(n_honest)]
    hs, st = impl.sign_batch([sks[o] for o in owner], hm)
    assert set(st) == {0}
    items = [(hpk[o], m, s, 0) for o, m, s in zip(owner, hm, hs)]
    step = max(1, n_honest // len(pks))
    for k, case in enumerate(zip(pks, msgs, sigs, want)):
        items.insert(min(len(items), k * (step + 1) + 3), case)
    return [list(x) for x in zip(*items)]


@pytest.mark.parametrize("mode", ["auto", "single", "lanes", "quads", "octets"])
def test_small_order_batch_verify_every_layout(impl, so, mode):
    from charon_amd.tbls import PAIR_AUTO, PAIR_LANES, PAIR_OCTETS, PAIR_QUADS, PAIR_SINGLE
    m = {"auto": PAIR_AUTO, "single": PAIR_SINGLE, "lanes": PAIR_LANES, "quads": PAIR_QUADS,
         "octets": PAIR_OCTETS}[mode]
    pks, msgs, sigs, want = _cases(so)
    prev = impl.set_pair_mode(m)
    try:
        assert impl.batch_verify_status(pks, msgs, sigs) == want
        if mode in ("auto", "octets"):
            # one case per call: AUTO takes the sixteen-lane check (verify_hex.hip) at n <= 4, OCTETS the octet one,
            # both raced by replicas
            for p, msg, s, w in zip(pks, msgs, sigs, want):
                assert impl.batch_verify_status([p], [msg], [s]) == [w]
        # the same cases at odd positions of a larger batch (pairs straddling wave edges)
        P, M, S, W = _padded(impl, so, 200, 1)
        assert impl.batch_verify_status(P, M, S) == W
    finally:
        impl.set_pair_mode(prev)


def test_small_order_queue_and_key_table(impl, so):
    pks, msgs, sigs, want = _cases(so)
    assert [impl.verify_queued(p, m, s) for p, m, s in zip(pks, msgs, sigs)] == want
    table = list(dict.fromkeys(pks))
    tst = impl.load_pubshares(table)
    # a key with cofactor torsion fails the table's subgroup test, exactly like Verify's decode
    assert [tst[table.index(p)] for p in pks] == [1 if w == 1 else 0 for w in want]
    pos = {p: j for j, p in enumerate(table)}
    assert impl.batch_verify_keys_status([pos[p] for p in pks], msgs, sigs) == want


@pytest.mark.parametrize("rlc_mode", ["windows", "batch", "auto"])
def test_small_order_rlc_every_path(impl, so, rlc_mode):
    """RLC windows (the window fails, the fallback decides), the batch-wide Pippenger check (it fails, windows decide)
    and AUTO; wire-format keys and the key table; statuses == per-item Verify == the oracle."""
    from charon_amd.tbls import RLC_AUTO, RLC_BATCH, RLC_WINDOWS
    m = {"windows": RLC_WINDOWS, "batch": RLC_BATCH, "auto": RLC_AUTO}[rlc_mode]
    P, M, S, W = _padded(impl, so, 1200, 2)
    prev = impl.set_rlc_mode(m)
    try:
        for seed in (bytes(32), os.urandom(32)):
            assert impl.batch_verify_rlc_status(P, M, S, seed=seed) == W
        table = list(dict.fromkeys(P))
        impl.load_pubshares(table)
        pos = {p: j for j, p in enumerate(table)}
        assert impl.batch_verify_rlc_keys_status([pos[p] for p in P], M, S) == W
    finally:
        impl.set_rlc_mode(prev)


def test_small_order_fav_and_aggregate(impl, so):
    """FastAggregateVerify with a small-order signature: status 2 (the signature is deserialized first,
    herumi.go:315-339); with a small-order key among honest ones: status 1.  Aggregate accepts any curve point only
    if it deserializes, so a small-order signature fails the whole call with the deserialization error."""
    from charon_amd.tbls import TBLSError
    c = so["verify"]
    sk, pk, msg = h(so["sk"]), h(so["pk"]), h(so["msg"])
    sig = impl.sign(sk, msg)
    small_sig = h(c[0]["sig"])
    small_pk = h(c[16]["pk"])
    groups = [([pk], sig, msg), ([pk], small_sig, msg), ([pk, small_pk], sig, msg), ([pk], h(c[4]["sig"]), msg)]
    assert impl.batch_verify_aggregate_status(groups) == [0, 2, 1, 2]
    with pytest.raises(TBLSError, match="cannot unmarshal signature into Herumi signature"):
        impl.aggregate([sig, small_sig])


def test_small_order_threshold_aggregate(impl, so):
    from charon_amd.tbls import TBLSError
    groups = [{int(k): h(v) for k, v in g["parts"].items()} for g in so["threshold_aggregate"]]
    res = impl.batch_threshold_aggregate(groups)
    for g, r in zip(so["threshold_aggregate"][:-1], res[:-1]):
        assert isinstance(r, TBLSError) and str(r) == "cannot unmarshal signature into Herumi signature", g["note"]
    assert res[-1] == h(so["threshold_aggregate"][-1]["out"])
    # fused with the aggregate Verify (core/sigagg): the aggregation status is carried into the verify status
    n = len(groups)
    res2, vst = impl.batch_threshold_aggregate_verify(groups, [h(so["pk"])] * n, [h(so["msg"])] * n)
    assert [str(r) if isinstance(r, TBLSError) else r for r in res2] == \
        [str(r) if isinstance(r, TBLSError) else r for r in res]
    assert vst[:-1] == [2] * (n - 1)
    # the honest 2-of-3 aggregate is of a different secret than so["pk"]: it must fail Verify, not pass
    assert vst[-1] == 3


def test_small_order_signed_data(impl, so):
    """eth2util/signing.Verify: the signing root is SHA-256(object_root || domain) on the GPU; a small-order
    signature fails deserialization (2) before the pairing; the all-zero rule does not apply to it."""
    from oracle import ssz
    pks, _, sigs, want = _cases(so)
    objs = [bytes([k]) * 32 for k in range(len(pks))]
    domain = ssz.compute_domain(bytes.fromhex("01000000"), bytes.fromhex("00001020"))
    got = impl.verify_signed_data_status(pks, objs, [domain] * len(pks), sigs)
    assert got[:24] == want[:24]
