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
