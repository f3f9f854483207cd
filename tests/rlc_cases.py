"""Inputs for RLC BatchVerify parity tests (host build and GPU): validator-shaped batches where all
partials of one validator share a signing root, plus the fixture cases with one message each.

The expected bitmap is always the per-item tbls.Verify outcome (oracle/bls12381.py statuses for the
fixtures, construction-known for the generated batches): random-linear-combination batching must
never change an item's result.
"""
import json
import os
import random

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
HERE = os.path.dirname(os.path.abspath(__file__))


def message_table(msgs_per_item):
    """Distinct-message table + per-item index (first-seen order), as a charon batcher builds it."""
    idx, table, pos = [], [], {}
    for m in msgs_per_item:
        if m not in pos:
            pos[m] = len(table)
            table.append(m)
        idx.append(pos[m])
    return table, idx


def fixture_batch():
    with open(os.path.join(HERE, "golden", "fixtures.json")) as f:
        fx = json.load(f)["verify"]
    pks = [bytes.fromhex(c["pk"]) for c in fx]
    msgs = [bytes.fromhex(c["msg"]) for c in fx]
    sigs = [bytes.fromhex(c["sig"]) for c in fx]
    return pks, msgs, sigs, [c["status"] for c in fx]


def validator_batch(sign, sk_to_pk, n_validators, shares_per_validator, seed, bad=()):
    """n_validators DVs x shares partials, one root per DV, items grouped by DV.
    bad: item indices to corrupt (cycling wrong root / swapped share / flipped bit).
    Returns pks, msgs, sigs, expected (0 = valid, None = known invalid: 2 or 3 depending on encoding)."""
    rng = random.Random(seed)
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(n_validators * shares_per_validator)]
    pk_of = [sk_to_pk(s) for s in sks]
    roots = [rng.randbytes(32) for _ in range(n_validators)]
    pks, msgs, sigs = [], [], []
    for v in range(n_validators):
        for s in range(shares_per_validator):
            k = v * shares_per_validator + s
            pks.append(pk_of[k])
            msgs.append(roots[v])
            sigs.append(sign(sks[k], roots[v]))
    expected = [0] * len(pks)
    for j, i in enumerate(sorted(bad)):
        kind = j % 3
        if kind == 0:    # signature over another root: same message slot, wrong content
            sigs[i] = sign(sks[i], rng.randbytes(32))
            expected[i] = 3
        elif kind == 1:  # another validator's pubshare
            pks[i] = pk_of[(i + shares_per_validator) % len(pk_of)]
            expected[i] = 3
        else:            # flipped bit in the signature (bad encoding or wrong point)
            b = bytearray(sigs[i])
            b[40] ^= 0x04
            sigs[i] = bytes(b)
            expected[i] = None
    return pks, msgs, sigs, expected
