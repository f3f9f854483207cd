"""GPU tests added in round 6.

* The two reference-held herumi vector sets round 5 left unused, through the product's batch
  entry points, batched and one item per call (AUTO then takes the sixteen-lane check, verify_hex.hip):
  - cluster/manifest/testdata/lock2.json: FastAggregateVerify of its aggregate over 12 pubshares on lock_hash
    (hipbls_verify_aggregate_batch);
  - cluster/manifest/testdata/lock.json: the DKG's threshold-aggregated deposit signatures under the DV keys
    (hipbls_verify_batch), next to the four cluster/examples locks and the deposit golden.
* The library loaded is the one built from the shipped sources (hipbls_build_id).
"""
import pytest

from oracle import ssz

pytestmark = pytest.mark.gpu


def h(s):
    return bytes.fromhex(s)


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def _lock2(kat):
    m = kat["manifest"]["lock2"]
    return [h(s) for s in m["public_shares"]], h(m["signature_aggregate"]), h(m["lock_hash"])


def _deposits(kat):
    m = kat["manifest"]["lock_deposits"]
    domain = ssz.compute_domain(ssz.DOMAIN_DEPOSIT, h(m["fork_version"]))
    pks, roots, sigs = [], [], []
    for dd in m["deposit_data"]:
        pks.append(h(dd["pubkey"]))
        roots.append(ssz.signing_data_root(ssz.deposit_message_root(h(dd["pubkey"]), h(dd["withdrawal_credentials"]),
                                                                    dd["amount"]), domain))
        sigs.append(h(dd["signature"]))
    return pks, roots, sigs


def test_manifest_lock2_fast_aggregate_verify(impl, kat):
    pks, sig, msg = _lock2(kat)
    groups = [(pks, sig, msg), (pks[1:], sig, msg), (pks, sig, msg[::-1]), (pks[::-1], sig, msg)]
    want = [0, 3, 3, 0]  # a key missing or another message fails; key order does not matter
    assert impl.batch_verify_aggregate_status(groups) == want  # one call, the sixteen-lane layout (<= 16 groups)
    for g, w in zip(groups, want):
        assert impl.batch_verify_aggregate_status([g]) == [w]  # one group per call
    # beside the four cluster/examples locks, in one call of 5 groups and in one of 20 (the octet layout)
    ex = [([h(s) for v in lk["validators"] for s in v["public_shares"]], h(lk["signature_aggregate"]),
           h(lk["lock_hash"])) for lk in kat["locks"]]
    assert impl.batch_verify_aggregate_status(ex + [groups[0]]) == [0] * 5
    assert impl.batch_verify_aggregate_status((ex + groups) * 2) == ([0] * 4 + want) * 2
    impl.verify_aggregate(pks, sig, msg)  # the single tbls.VerifyAggregate entry point


def test_manifest_lock_deposit_signatures(impl, kat):
    pks, roots, sigs = _deposits(kat)
    assert impl.batch_verify_status(pks, roots, sigs) == [0, 0]
    assert impl.batch_verify_status(pks, roots[::-1], sigs) == [3, 3]  # each other's deposit message
    for pk, root, sig in zip(pks, roots, sigs):
        assert impl.batch_verify_status([pk], [root], [sig]) == [0]  # one item per call: sixteen lanes
        assert impl.batch_verify_status([pk], [root[::-1]], [sig]) == [3]
    # with the deposit golden's signatures (eth2util/deposit) in one mixed batch
    dk = kat["deposit"]
    from oracle import bls12381 as bls
    gp, gr, gs = [], [], []
    domain = ssz.compute_domain(ssz.DOMAIN_DEPOSIT, h("00001020"))
    for sk in dk["sks"]:
        pk = bls.secret_to_public_key(h(sk))
        e = {x["pubkey"]: x for x in dk["entries"]}[pk.hex()]
        gp.append(pk)
        gr.append(ssz.signing_data_root(ssz.deposit_message_root(pk, h(e["withdrawal_credentials"]), e["amount"]),
                                        domain))
        gs.append(h(e["signature"]))
    assert impl.batch_verify_status(pks + gp, roots + gr, sigs + gs) == [0] * (2 + len(gp))


def test_loaded_library_is_the_shipped_sources(impl):
    from charon_amd import build
    from charon_amd.tbls import build_id
    assert build_id() == {"src": build.source_digest(), "flags": build.flags_digest()}


# ---------------------------------------------------------------- fuzzed encodings (round 6)
def _mutations(rng, valid, size, p):
    """Structured encodings around `valid` points (size 48: G1, 96: G2): random x below p with random flags, the
    valid points negated (sign bit), one random bit flipped (flags included for some), x = p, p + 1, 2^381 - 1, x = 0,
    and the infinity encodings with stray bits."""
    out = []
    for _ in range(150):
        b = bytearray(rng.randbytes(size))
        for k in range(0, size, 48):  # each 48-byte coordinate below p
            x = int.from_bytes(b[k:k + 48], "big") & ((1 << 381) - 1)
            b[k:k + 48] = (x % p).to_bytes(48, "big")
        b[0] |= 0x80 | (0x20 if rng.random() < 0.5 else 0)
        out.append(bytes(b))
    for v in valid:
        b = bytearray(v)
        b[0] ^= 0x20
        out.append(bytes(b))  # the negated point: still valid
        b = bytearray(v)
        bit = rng.randrange(8 * size) if rng.random() < 0.2 else rng.randrange(3, 8 * size)  # a flag bit in 20 %
        b[bit // 8] ^= 0x80 >> (bit % 8)
        out.append(bytes(b))
    top = [p, p + 1, (1 << 381) - 1, 0]
    for x in top:
        enc = bytearray(x.to_bytes(48, "big") + bytes(size - 48))
        enc[0] |= 0x80
        out.append(bytes(enc))
        if size == 96:
            enc = bytearray(bytes(48) + x.to_bytes(48, "big"))
            enc[0] |= 0x80
            out.append(bytes(enc))
    inf = bytearray(size)
    inf[0] = 0xC0
    out.append(bytes(inf))
    for flags in (0x40, 0xE0, 0x00, 0xA0):
        b = bytearray(size)
        b[0] = flags
        out.append(bytes(b))
    b = bytearray(inf)
    b[-1] = 1
    out.append(bytes(b))
    return out


def test_fuzzed_encodings_deserialize_like_the_oracle(impl):
    """herumi Deserialize per point (hipbls_deserialize_status) equals the oracle's decompression on ~700 structured
    encodings: random x with random flags (both square and non-square x, off-subgroup points), negated valid points,
    single bit flips, x >= p, x = 0 and the infinity encodings with stray bits (SURVEY 8a edge list)."""
    import random

    from oracle import bls12381 as bls
    rng = random.Random(606)
    sks = [rng.randrange(1, bls.R).to_bytes(32, "big") for _ in range(60)]
    pks = [bls.secret_to_public_key(sk) for sk in sks]
    sigs = [bls.sign(sk, b"fuzz %d" % i) for i, sk in enumerate(sks[:40])]
    g1 = _mutations(rng, pks, 48, bls.P)
    g2 = _mutations(rng, sigs, 96, bls.P)

    def ok(fn, b):
        try:
            fn(b)
            return True
        except bls.BLSError:
            return False

    want1 = [0 if ok(bls.g1_decompress, x) else 1 for x in g1]
    want2 = [0 if ok(bls.g2_decompress, x) else 2 for x in g2]
    assert impl.deserialize_status(g1, 1) == want1
    assert impl.deserialize_status(g2, 2) == want2
    assert 0 < want1.count(0) < len(want1) and 0 < want2.count(0) < len(want2)


def test_fuzzed_verify_items_match_the_oracle(impl):
    """Mixed Verify batches over valid and mutated keys, signatures and messages: the statuses equal the oracle's
    (decode order pk -> sig -> pairing, herumi.go:285-301), batched and one item per call."""
    import random

    from oracle import bls12381 as bls
    rng = random.Random(607)
    items = []
    for i in range(24):
        sk = rng.randrange(1, bls.R).to_bytes(32, "big")
        msg = rng.randbytes(32)
        pk, sig = bls.secret_to_public_key(sk), bls.sign(sk, msg)
        kind = i % 6
        if kind == 1:
            msg = msg[::-1]  # wrong message
        elif kind == 2:
            sig = bytes([sig[0] ^ 0x20]) + sig[1:]  # -sig: decodes, fails the pairing
        elif kind == 3:
            pk = bytes([pk[0]]) + bytes([pk[1] ^ 0x01]) + pk[2:]  # a flipped key bit
        elif kind == 4:
            sig = sig[:50] + bytes([sig[50] ^ 0x10]) + sig[51:]  # a flipped signature bit
        elif kind == 5:
            pk, sig = bls.secret_to_public_key(sk), bls.sign(sk, msg)  # valid, again
        items.append((pk, msg, sig))
    want = [bls.verify_status(pk, m, s) for pk, m, s in items]
    pks, msgs, sigs = zip(*items)
    assert impl.batch_verify_status(list(pks), list(msgs), list(sigs)) == want
    for (pk, m, s), w in zip(items[:12], want[:12]):
        assert impl.batch_verify_status([pk], [m], [s]) == [w]
    assert set(want) >= {0, 3}
