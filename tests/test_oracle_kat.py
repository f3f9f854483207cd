"""Pin the CPU oracle to every herumi-produced vector the reference's own tests hold.

The vectors live in tests/golden/kat_reference.json (made by tests/golden/make_kat_reference.py from
the reference's test files).  If the oracle passes these, its Sign/SecretToPublicKey/Verify/
FastAggregateVerify and the SSZ signing roots agree with herumi on honest inputs.
"""
import pytest

from oracle import bls12381 as bls
from oracle import ssz


def h(s):
    return bytes.fromhex(s)


def test_rfc9380_expand_message_vector():
    # RFC 9380 K.1 (expand_message_xmd SHA-256), msg = "", len_in_bytes = 0x20
    out = bls.expand_message_xmd(b"", b"QUUX-V01-CS02-with-expander-SHA256-128", 0x20)
    assert out.hex() == "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"


def test_rfc9380_hash_to_g2_vector():
    # RFC 9380 J.10.1 BLS12381G2_XMD:SHA-256_SSWU_RO_, msg = ""
    Q = bls.hash_to_g2(b"", b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_")
    assert Q[0][0] == 0x0141EBFBDCA40EB85B87142E130AB689C673CF60F1A3E98D69335266F30D9B8D4AC44C1038E9DCDD5393FAF5C41FB78A
    assert Q[0][1] == 0x05CB8437535E20ECFFAEF7752BADDF98034139C38452458BAEEFAB379BA13DFF5BF5DD71B72418717047F5B0F37DA03D


def test_generators_and_isogeny():
    assert bls.g1_on_curve(bls.G1_GEN) and bls.g2_on_curve(bls.G2_GEN)
    assert bls.g1_mul(bls.G1_GEN, bls.R) is None
    assert bls.g2_mul(bls.G2_GEN, bls.R) is None
    u = (12345, 67890)
    assert bls.g2_on_curve(bls.iso_map_g2(bls.map_to_curve_sswu(u)))


def test_prysm_attestation_kat(kat):
    k = kat["prysm"]
    sig = bls.sign(h(k["sk"]), h(k["signing_root"]))
    assert sig.hex() == k["sig"]
    pk = bls.secret_to_public_key(h(k["sk"]))
    assert bls.verify_status(pk, h(k["signing_root"]), sig) == 0
    assert bls.verify_status(pk, h(k["signing_root"])[::-1], sig) == 3


def test_teku_registration_kat(kat):
    k = kat["teku"]
    obj_root = ssz.validator_registration_root(h(k["fee_recipient"]), k["gas_limit"], k["timestamp"], h(k["pubkey"]))
    # beaconmock genesis fork version 0x00001020 (testutil/beaconmock/static.json)
    assert ssz.compute_domain(ssz.DOMAIN_APPLICATION_BUILDER, h("00001020")).hex() == k["domain"]
    root = ssz.signing_data_root(obj_root, h(k["domain"]))
    sig = bls.sign(h(k["sk"]), root)
    assert sig.hex() == k["sig"]
    assert bls.verify_status(bls.secret_to_public_key(h(k["sk"])), root, sig) == 0


def test_deposit_golden_kat(kat):
    k = kat["deposit"]
    by_pk = {e["pubkey"]: e for e in k["entries"]}
    domain = ssz.compute_domain(ssz.DOMAIN_DEPOSIT, h("00001020"))
    for sk in k["sks"]:
        pk = bls.secret_to_public_key(h(sk))
        e = by_pk[pk.hex()]
        mroot = ssz.deposit_message_root(pk, h(e["withdrawal_credentials"]), e["amount"])
        assert mroot.hex() == e["deposit_message_root"]
        sig = bls.sign(h(sk), ssz.signing_data_root(mroot, domain))
        assert sig.hex() == e["signature"]


@pytest.mark.parametrize("i", [0, 1, 2, 3])
def test_cluster_lock_fast_aggregate_verify(kat, i):
    lock = kat["locks"][i]
    pks = [h(s) for v in lock["validators"] for s in v["public_shares"]]
    bls.verify_aggregate(pks, h(lock["signature_aggregate"]), h(lock["lock_hash"]))
    with pytest.raises(bls.BLSError):
        bls.verify_aggregate(pks[:-1], h(lock["signature_aggregate"]), h(lock["lock_hash"]))


def test_cluster_lock_builder_registrations(kat):
    lock = kat["locks"][3]
    domain = ssz.compute_domain(ssz.DOMAIN_APPLICATION_BUILDER, h(lock["fork_version"]))
    n = 0
    for v in lock["validators"]:
        br = v["builder_registration"]
        obj = ssz.validator_registration_root(h(br["fee_recipient"]), br["gas_limit"], br["timestamp"], h(br["pubkey"]))
        root = ssz.signing_data_root(obj, domain)
        assert bls.verify_status(h(v["distributed_public_key"]), root, h(br["signature"])) == 0
        n += 1
    assert n == 3


def test_threshold_roundtrip_matches_sign():
    # tbls_test.go:73-98: ThresholdAggregate of t-of-n partials == Sign(secret)
    msg = b"hello obol!"
    secret = 0x1234567890ABCDEF
    shares = bls.threshold_split_poly(secret, [777, 999], 5)
    full = bls.sign(bls.sk_serialize(secret), msg)
    parts = {i: bls.sign(shares[i], msg) for i in (1, 3, 5)}
    assert bls.threshold_aggregate(parts) == full
    assert bls.recover_secret({i: shares[i] for i in (2, 4, 5)}) == bls.sk_serialize(secret)


def test_manifest_lock2_fast_aggregate_verify(kat):
    """cluster/manifest/testdata/lock2.json (load_test.go:77): its aggregate over the 12 pubshares on lock_hash."""
    m = kat["manifest"]["lock2"]
    pks = [h(s) for s in m["public_shares"]]
    assert len(pks) == 12
    bls.verify_aggregate(pks, h(m["signature_aggregate"]), h(m["lock_hash"]))
    with pytest.raises(bls.BLSError):
        bls.verify_aggregate(pks[1:], h(m["signature_aggregate"]), h(m["lock_hash"]))


def test_manifest_lock_deposit_signatures(kat):
    """cluster/manifest/testdata/lock.json (load_test.go:31): the DKG's threshold-aggregated deposit signatures verify
    under the DV keys over the deposit domain of fork 0x00001020."""
    m = kat["manifest"]["lock_deposits"]
    domain = ssz.compute_domain(ssz.DOMAIN_DEPOSIT, h(m["fork_version"]))
    assert len(m["deposit_data"]) == 2
    for dd in m["deposit_data"]:
        root = ssz.signing_data_root(ssz.deposit_message_root(h(dd["pubkey"]), h(dd["withdrawal_credentials"]),
                                                              dd["amount"]), domain)
        assert bls.verify_status(h(dd["pubkey"]), root, h(dd["signature"])) == 0
        assert bls.verify_status(h(dd["pubkey"]), root[::-1], h(dd["signature"])) == 3
