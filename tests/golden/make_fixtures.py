"""Generate tests/golden/fixtures.json with the CPU oracle (oracle/bls12381.py).

Inputs are seeded (random.Random(0x636861726f6e), the SURVEY §8d seed); expected outputs are the
oracle's, which is pinned to herumi by tests/test_oracle_kat.py.  Edge cases the reference does not
pin follow oracle/bls12381.py::EDGE_POLICY (parity for those is against the oracle's documented
choice, not herumi).
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12381 as bls  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures.json")
SEED = 0x636861726F6E


def non_subgroup_g2(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            pt = (x, y)
            assert bls.g2_mul(pt, bls.R) is not None
            return bls.g2_compress(pt)


def non_subgroup_g1(rng):
    while True:
        x = rng.randrange(bls.P)
        y = bls.fp_sqrt((x ** 3 + 4) % bls.P)
        if y is not None:
            pt = (x, y)
            assert bls.g1_mul(pt, bls.R) is not None
            return bls.g1_compress(pt)


def not_on_curve_g1(rng):
    while True:
        x = rng.randrange(bls.P)
        if bls.fp_sqrt((x ** 3 + 4) % bls.P) is None:
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def main():
    rng = random.Random(SEED)
    sks = [rng.randrange(1, bls.R).to_bytes(32, "big") for _ in range(6)]
    pks = [bls.secret_to_public_key(s) for s in sks]
    msgs = [rng.randbytes(32) for _ in range(6)] + [b"hello obol!", b"", bytes(range(100))]
    cases = []

    def add(pk, msg, sig, note):
        cases.append({"pk": pk.hex(), "msg": msg.hex(), "sig": sig.hex(),
                      "status": bls.verify_status(pk, msg, sig), "note": note})

    for i in range(6):
        add(pks[i], msgs[i], bls.sign(sks[i], msgs[i]), "valid")
    for j, m in enumerate(msgs[6:]):
        add(pks[j], m, bls.sign(sks[j], m), "valid, msg len %d" % len(m))
    s0 = bls.sign(sks[0], msgs[0])
    add(pks[0], msgs[1], s0, "wrong message")
    add(pks[1], msgs[0], s0, "wrong key")
    add(pks[0], msgs[0], bls.sign(sks[1], msgs[0]), "signature from another key")
    flipped = bytearray(s0)
    flipped[50] ^= 0x01
    add(pks[0], msgs[0], bytes(flipped), "flipped bit in signature x")
    sflag = bytearray(s0)
    sflag[0] ^= 0x20
    add(pks[0], msgs[0], bytes(sflag), "sign flag flipped (=-sigma)")
    nc = bytearray(s0)
    nc[0] &= 0x7F
    add(pks[0], msgs[0], bytes(nc), "signature missing compression flag")
    pnc = bytearray(pks[0])
    pnc[0] &= 0x7F
    add(bytes(pnc), msgs[0], s0, "pubkey missing compression flag")
    big = bytearray((bls.P + 5).to_bytes(48, "big"))
    big[0] |= 0x80
    add(bytes(big), msgs[0], s0, "pubkey x >= p")
    bigs = bytearray((bls.P).to_bytes(48, "big") + bytes(48))
    bigs[0] |= 0x80
    add(pks[0], msgs[0], bytes(bigs), "signature x_c1 = p")
    add(bls.g1_compress(None), msgs[0], s0, "pubkey infinity")
    add(pks[0], msgs[0], bls.g2_compress(None), "signature infinity")
    inf_garbage = bytearray(bls.g1_compress(None))
    inf_garbage[10] = 1
    add(bytes(inf_garbage), msgs[0], s0, "pubkey infinity flag with payload")
    add(pks[0], msgs[0], bytes(96), "all-zero signature")
    add(bytes(48), msgs[0], s0, "all-zero pubkey")
    add(non_subgroup_g1(rng), msgs[0], s0, "pubkey on curve, not in G1")
    add(pks[0], msgs[0], non_subgroup_g2(rng), "signature on curve, not in G2")
    add(not_on_curve_g1(rng), msgs[0], s0, "pubkey x not on curve")

    # threshold aggregation groups (tbls_test.go:73-98 shape, plus error cases)
    tagg = []
    msg = b"hello obol!"

    def add_group(parts, note):
        try:
            out = bls.threshold_aggregate(parts).hex()
            err = None
        except bls.BLSError as e:
            out, err = None, str(e)
        tagg.append({"parts": {str(k): v.hex() for k, v in parts.items()}, "out": out, "err": err, "note": note})

    for (n, t) in [(5, 3), (6, 4), (10, 7), (1, 1), (4, 2)]:
        secret = rng.randrange(1, bls.R)
        shares = bls.threshold_split_poly(secret, [rng.randrange(bls.R) for _ in range(t - 1)], n)
        ids = sorted(rng.sample(range(1, n + 1), t))
        parts = {i: bls.sign(shares[i], msg) for i in ids}
        add_group(parts, "%d-of-%d" % (t, n))
        assert bls.threshold_aggregate(parts) == bls.sign(bls.sk_serialize(secret), msg)
    good = {1: bls.sign(sks[0], msg), 2: bls.sign(sks[1], msg)}
    add_group({0: good[1], 2: good[2]}, "id 0")
    bad = dict(good)
    bad[2] = bytes(96)
    add_group(bad, "undecodable partial")
    add_group({1: good[1], 2: non_subgroup_g2(rng)}, "partial not in G2")

    small = small_order_cases(random.Random(SEED + 13))

    with open(OUT, "w") as f:
        json.dump({"seed": SEED, "verify": cases, "threshold_aggregate": tagg, "small_order": small}, f, indent=1)
    print("wrote %s: %d verify, %d tagg, %d small-order" % (OUT, len(cases), len(tagg), len(small["verify"])))


# ---------------------------------------------------------------- points of small order (cofactor torsion)
# Verify decides the signature's G2 membership from its own Miller loop (charon_amd/csrc/pairing.h
# g2_subgroup_from_miller): the loop runs T over |x|'s bits from T = sig, and a point of small order makes a doubling
# or addition step exceptional (Z = 0).  herumi rejects such a signature at deserialization (tbls/herumi.go:291-294),
# status 2, whatever the key.  These cases pin that on every device layout.  Public keys of small order (G1 cofactor
# torsion: orders 3 and 11) exercise the phi subgroup test the same way (herumi.go:286-289, status 1).
X = -bls.X_ABS
H1 = (X - 1) ** 2 // 3
H2 = (X ** 8 - 4 * X ** 7 + 5 * X ** 6 - 4 * X ** 4 + 6 * X ** 3 - 4 * X ** 2 - 4 * X + 13) // 9


def _rand_g2(rng):
    while True:
        px = (rng.randrange(bls.P), rng.randrange(bls.P))
        py = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(px), px), bls.B2))
        if py is not None:
            return (px, py)


def _rand_g1(rng):
    while True:
        px = rng.randrange(bls.P)
        py = bls.fp_sqrt((px ** 3 + 4) % bls.P)
        if py is not None:
            return (px, py)


def _of_order(rng, q, n_total, rand_pt, mul):
    """A point of order exactly q: the q-primary part of a random point, multiplied down to order q."""
    m = n_total
    while m % q == 0:
        m //= q
    while True:
        pt = mul(rand_pt(rng), m)
        if pt is None:
            continue
        while mul(pt, q) is not None:
            pt = mul(pt, q)
        assert mul(pt, q) is None
        return pt


def small_order_cases(rng):
    sks = [rng.randrange(1, bls.R).to_bytes(32, "big") for _ in range(2)]
    pks = [bls.secret_to_public_key(s) for s in sks]
    msgs = [rng.randbytes(32) for _ in range(2)]
    sig = bls.sign(sks[0], msgs[0])
    sig_pt = bls.g2_decompress(sig)
    pk_pt = bls.g1_decompress(pks[0])
    inf_pk = bls.g1_compress(None)
    sigs, pkeys = [], []
    for q in (13, 23):
        s = _of_order(rng, q, H2 * bls.R, _rand_g2, bls.g2_mul)
        sigs.append((bls.g2_compress(s), "signature of order %d" % q))
        sigs.append((bls.g2_compress(bls.g2_add(sig_pt, s)), "honest signature + order-%d point" % q))
    for q in (3, 11):
        p = _of_order(rng, q, H1 * bls.R, _rand_g1, bls.g1_mul)
        pkeys.append((bls.g1_compress(p), "public key of order %d" % q))
        pkeys.append((bls.g1_compress(bls.g1_add(pk_pt, p)), "public key + order-%d point" % q))
    cases = []

    def add(pk, msg, s, note):
        cases.append({"pk": pk.hex(), "msg": msg.hex(), "sig": s.hex(), "status": bls.verify_status(pk, msg, s),
                      "note": note})

    for s, note in sigs:
        add(pks[0], msgs[0], s, note + ", signer's key")
        add(pks[0], msgs[1], s, note + ", wrong message")
        add(pks[1], msgs[0], s, note + ", other key")
        add(inf_pk, msgs[0], s, note + ", infinity key")
    for p, note in pkeys:
        add(p, msgs[0], sig, note + ", honest signature")
        add(p, msgs[0], sigs[0][0], note + ", order-13 signature")
    add(pks[0], msgs[0], sig, "honest control")
    assert [c["status"] for c in cases[:16]] == [2] * 16 and [c["status"] for c in cases[16:24]] == [1] * 8
    # threshold aggregation with a small-order partial (herumi deserializes every partial first: status 2)
    secret = rng.randrange(1, bls.R)
    shares = bls.threshold_split_poly(secret, [rng.randrange(bls.R)], 3)
    parts = {i: bls.sign(shares[i], msgs[0]) for i in (1, 2)}
    tagg = [{"parts": {"1": parts[1].hex(), "2": s.hex()}, "note": note} for s, note in sigs]
    tagg.append({"parts": {str(k): v.hex() for k, v in parts.items()}, "note": "honest 2-of-3",
                 "out": bls.threshold_aggregate(parts).hex()})
    return {"verify": cases, "threshold_aggregate": tagg, "msg": msgs[0].hex(), "sk": sks[0].hex(),
            "pk": pks[0].hex()}


if __name__ == "__main__":
    main()
