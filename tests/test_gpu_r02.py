"""GPU parity and boundary tests added in round 2 (VERDICT r01 "Next round" items 1, 3, 7, 8):

* Aggregate([]) and share ids as Fr elements, pinned to the reference's semantics
  (/root/reference/tbls/herumi.go:220-242, 264-271) and to the oracle;
* the RLC cancellation cases that only the random scalars catch;
* full-size C2 (65,536 Verify) and C3 (10,000 x 7-of-10) runs with oracle-checked samples;
* a 512-key FastAggregateVerify negative case against the oracle;
* the submission queue (coalesced n = 1 Verify from many threads), cross-stream workspace ordering,
  the resident H(m) cache, GPU signing roots, and the cluster-lock bulk verification.

Every check is bit-exact against the oracle or against construction-known outcomes.
"""
import os
import random
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def h(s):
    return bytes.fromhex(s)


@pytest.fixture(scope="module")
def impl():
    from charon_amd.tbls import HipBLS
    return HipBLS()


def _keys(impl, rng, n):
    sks = [rng.randrange(1, R_ORDER).to_bytes(32, "big") for _ in range(n)]
    pks, st = impl.secret_to_public_key_batch(sks)
    assert set(st) <= {0}
    return sks, pks


# ---------------------------------------------------------------- Aggregate (herumi.go:220-242)
def test_aggregate_empty_is_infinity_no_error(impl):
    from charon_amd.tbls import INFINITY_G2
    from oracle import bls12381 as bls
    assert impl.aggregate([]) == INFINITY_G2 == bls.aggregate([])


def test_aggregate_parallel_vs_oracle_and_property(impl):
    from charon_amd.tbls import TBLSError
    from oracle import bls12381 as bls
    rng = random.Random(5)
    msg = rng.randbytes(32)
    sks, _ = _keys(impl, rng, 2000)
    sigs, st = impl.sign_batch(sks, [msg] * len(sks))
    assert set(st) == {0}
    # oracle on a prefix (pure-Python decompressions are slow)
    assert impl.aggregate(sigs[:40]) == bls.aggregate(sigs[:40])
    # whole set: sum_i sk_i H(m) == (sum_i sk_i) H(m), an independent Sign
    total = sum(int.from_bytes(s, "big") for s in sks) % R_ORDER
    assert impl.aggregate(sigs) == impl.sign(total.to_bytes(32, "big"), msg)
    # an infinity signature contributes nothing; a bad encoding anywhere fails the call
    assert impl.aggregate(sigs[:3] + [b"\xc0" + bytes(95)]) == impl.aggregate(sigs[:3])
    bad = bytearray(sigs[1500])
    bad[0] &= 0x7F
    with pytest.raises(TBLSError, match="cannot unmarshal signature into Herumi signature"):
        impl.aggregate(sigs[:1500] + [bytes(bad)] + sigs[1501:])


# ---------------------------------------------------------------- share ids as Fr (herumi.go:264-271)
def _shares_at(secret, tail, ids):
    """share(id) = f(id mod r) for f = secret + tail_1 x + ...: what SetDecString(strconv.Itoa(id)) implies."""
    out = {}
    for i in ids:
        x = i % R_ORDER
        acc = 0
        for c in reversed([secret] + tail):
            acc = (acc * x + c) % R_ORDER
        out[i] = acc.to_bytes(32, "big")
    return out


@pytest.mark.parametrize("ids", [(-3, 5, 2 ** 40 + 1), (-(2 ** 63), 2 ** 63 - 1, 7), (2 ** 32 + 1, 1, -1)])
def test_threshold_aggregate_signed_and_large_ids(impl, ids):
    from oracle import bls12381 as bls
    rng = random.Random(sum(ids) & 0xFFFF)
    secret = rng.randrange(1, R_ORDER)
    tail = [rng.randrange(R_ORDER) for _ in range(len(ids) - 1)]
    shares = _shares_at(secret, tail, ids)
    msg = rng.randbytes(32)
    sigs, st = impl.sign_batch([shares[i] for i in ids], [msg] * len(ids))
    assert set(st) == {0}
    parts = dict(zip(ids, sigs))
    got = impl.threshold_aggregate(parts)
    assert got == bls.threshold_aggregate(parts) == impl.sign(secret.to_bytes(32, "big"), msg)
    assert impl.recover_secret(shares) == bls.recover_secret(shares) == secret.to_bytes(32, "big")


def test_threshold_aggregate_id_zero_and_truncation(impl):
    """id 0 cannot combine (oracle and engine agree); 2^32 + 1 is NOT id 1 (no uint32 truncation)."""
    from charon_amd.tbls import TBLSError
    from oracle import bls12381 as bls
    rng = random.Random(77)
    secret = rng.randrange(1, R_ORDER)
    tail = [rng.randrange(R_ORDER)]
    msg = rng.randbytes(32)
    sh = _shares_at(secret, tail, (1, 2, 2 ** 32 + 1))
    sigs, _ = impl.sign_batch([sh[1], sh[2], sh[2 ** 32 + 1]], [msg] * 3)
    res = impl.batch_threshold_aggregate([{0: sigs[0], 2: sigs[1]}, {2 ** 32 + 1: sigs[2], 2: sigs[1]}])
    assert isinstance(res[0], TBLSError) and str(res[0]) == "cannot combine signatures"
    with pytest.raises(bls.BLSError, match="cannot combine signatures"):
        bls.threshold_aggregate({0: sigs[0], 2: sigs[1]})
    assert res[1] == impl.sign(secret.to_bytes(32, "big"), msg)
    # the same partial labelled 1 instead of 2^32 + 1 gives a different (wrong) aggregate
    assert impl.threshold_aggregate({1: sigs[2], 2: sigs[1]}) != res[1]


# ---------------------------------------------------------------- RLC: what the random scalars are for
def test_rlc_cancellation_cases(impl):
    """Two items under one root with swapped signatures, and a (sig_i + D, sig_j - D) pair: a plain
    (unrandomized) sum accepts both; the RLC bitmap must equal per-item Verify (status 3)."""
    from oracle import bls12381 as bls
    rng = random.Random(2024)
    sks, pks = _keys(impl, rng, 16)
    root = rng.randbytes(32)
    other = rng.randbytes(32)
    sigs, _ = impl.sign_batch(sks, [root] * 8 + [other] * 8)
    msgs = [root] * 8 + [other] * 8
    sigs = list(sigs)
    sigs[1], sigs[2] = sigs[2], sigs[1]  # swapped within one root: sum unchanged
    d = bls.g2_mul(bls.hash_to_g2(b"delta"), 12345)
    s5, s6 = bls.g2_decompress(sigs[5]), bls.g2_decompress(sigs[6])
    sigs[5] = bls.g2_compress(bls.g2_add(s5, d))
    sigs[6] = bls.g2_compress(bls.g2_add(s6, bls.g2_neg(d)))
    want = impl.batch_verify_status(pks, msgs, sigs)
    assert want == [0, 3, 3, 0, 0, 3, 3, 0] + [0] * 8
    for seed in (bytes(32), b"\x01" * 32, os.urandom(32)):
        assert impl.batch_verify_rlc_status(pks, msgs, sigs, seed=seed) == want
    # same with the pubshare table
    assert impl.load_pubshares(pks) == [0] * 16
    assert impl.batch_verify_rlc_keys_status(list(range(16)), msgs, sigs) == want


# ---------------------------------------------------------------- full-size configs with oracle samples
def test_c2_full_size_with_oracle_sample(impl):
    """BASELINE configs[1]: 65,536 Verify over distinct roots, 1% corrupted; a seeded 32-item sample
    (corrupted items included) is checked against oracle/bls12381.py, the rest by construction."""
    from oracle import bls12381 as bls
    rng = random.Random(0xC2)
    n = 65536
    sks, pks = _keys(impl, rng, 512)
    owner = [rng.randrange(512) for _ in range(n)]
    roots = [rng.randbytes(32) for _ in range(n)]
    sigs, st = impl.sign_batch([sks[o] for o in owner], roots)
    assert set(st) == {0}
    pk_list = [pks[o] for o in owner]
    bad = sorted(rng.sample(range(n), n // 100))
    sigs = list(sigs)
    for j, i in enumerate(bad):
        if j % 3 == 0:
            roots[i] = roots[i][::-1]
        elif j % 3 == 1:
            pk_list[i] = pks[(owner[i] + 1) % 512]
        else:
            b = bytearray(sigs[i])
            b[40] ^= 0x04
            sigs[i] = bytes(b)
    got = impl.batch_verify_status(pk_list, roots, sigs)
    assert {i for i, s in enumerate(got) if s != 0} == set(bad)
    sample = sorted(rng.sample(range(n), 24)) + bad[:8]
    for i in sample:
        assert got[i] == bls.verify_status(pk_list[i], roots[i], sigs[i]), i


def test_c3_full_size_aggregates(impl):
    """BASELINE configs[2]: 10,000 validators x a random 7-of-10 subset; every aggregate must equal
    Sign(secret) byte for byte (tbls_test.go:73-98) and verify under the validator key; 6 groups are
    recomputed by the oracle."""
    from oracle import bls12381 as bls
    rng = random.Random(0xC3)
    G, t, nsh = 10000, 7, 10
    secrets_ = [rng.randrange(1, R_ORDER) for _ in range(G)]
    roots = [rng.randbytes(32) for _ in range(G)]
    part_sks, part_msgs, groups_ids = [], [], []
    for g in range(G):
        poly = [secrets_[g]] + [rng.randrange(R_ORDER) for _ in range(t - 1)]
        ids = sorted(rng.sample(range(1, nsh + 1), t))
        groups_ids.append(ids)
        for i in ids:
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % R_ORDER
            part_sks.append(acc.to_bytes(32, "big"))
            part_msgs.append(roots[g])
    psigs, st = impl.sign_batch(part_sks, part_msgs)
    assert set(st) == {0}
    groups, k = [], 0
    for g in range(G):
        groups.append({i: psigs[k + j] for j, i in enumerate(groups_ids[g])})
        k += t
    aggs = impl.batch_threshold_aggregate(groups)
    full, st = impl.sign_batch([s.to_bytes(32, "big") for s in secrets_], roots)
    assert set(st) == {0}
    assert aggs == full
    dv_pks, _ = impl.secret_to_public_key_batch([s.to_bytes(32, "big") for s in secrets_])
    assert impl.batch_verify_status(dv_pks, roots, aggs) == [0] * G
    for g in rng.sample(range(G), 6):
        assert bls.threshold_aggregate(groups[g]) == aggs[g]


def test_fav_512_negative_vs_oracle(impl):
    """Sync-committee FastAggregateVerify over 512 keys: honest, wrong root, one key swapped, one key
    missing -- one launch; the swapped-key case is recomputed by the oracle."""
    from oracle import bls12381 as bls
    rng = random.Random(512)
    sks, pks = _keys(impl, rng, 513)
    root = rng.randbytes(32)
    sigs, _ = impl.sign_batch(sks[:512], [root] * 512)
    agg = impl.aggregate(sigs)
    swapped = pks[:511] + [pks[512]]
    groups = [(pks[:512], agg, root), (pks[:512], agg, root[::-1]), (swapped, agg, root), (pks[:511], agg, root)]
    assert impl.batch_verify_aggregate_status(groups) == [0, 3, 3, 3]
    with pytest.raises(bls.BLSError, match="signature verification failed"):
        bls.verify_aggregate(swapped, agg, root)


# ---------------------------------------------------------------- submission queue
def _mixed_items(impl, n, seed):
    rng = random.Random(seed)
    sks, pks = _keys(impl, rng, 32)
    owner = [rng.randrange(32) for _ in range(n)]
    msgs = [rng.randbytes(32) for _ in range(n)]
    sigs, _ = impl.sign_batch([sks[o] for o in owner], msgs)
    pk_list = [pks[o] for o in owner]
    sigs = list(sigs)
    for i in range(0, n, 7):
        msgs[i] = msgs[i][::-1]
    for i in range(3, n, 11):
        b = bytearray(sigs[i])
        b[0] &= 0x7F
        sigs[i] = bytes(b)
    return pk_list, msgs, sigs


def test_queue_concurrent_single_verifies_equal_batch(impl):
    """64 host threads each doing synchronous n = 1 Verify calls (tbls.Verify from many goroutines):
    statuses equal the batch call, and the calls are coalesced into fewer launches."""
    pks, msgs, sigs = _mixed_items(impl, 64 * 4, 3)
    want = impl.batch_verify_status(pks, msgs, sigs)
    impl.queue_config(65536, 500)
    b0, i0 = impl.queue_stats()
    got = [None] * len(pks)

    def worker(t):
        for i in range(t, len(pks), 64):
            got[i] = impl.verify_queued(pks[i], msgs[i], sigs[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    b1, i1 = impl.queue_stats()
    assert got == want
    assert i1 - i0 == len(pks)
    assert b1 - b0 < len(pks) // 8, (b1 - b0, len(pks))


def test_queue_async_in_flight_throughput(impl):
    """64 threads keep 64 submissions each in flight (4,096 outstanding n = 1 Verify calls): statuses
    equal the batch call; the sustained rate is printed (coalesced batches, no lock held across the GPU run)."""
    n = 64 * 64 * 4
    pks, msgs, sigs = _mixed_items(impl, n, 4)
    want = impl.batch_verify_status(pks, msgs, sigs)
    impl.queue_config(65536, 200)
    got = [None] * n
    b0, _ = impl.queue_stats()

    def worker(t):
        mine = list(range(t, n, 64))
        for k in range(0, len(mine), 64):
            chunk = mine[k:k + 64]
            tickets = [impl.verify_submit(pks[i], msgs[i], sigs[i]) for i in chunk]
            for i, tk in zip(chunk, tickets):
                got[i] = impl.verify_wait(tk)

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    b1, _ = impl.queue_stats()
    assert got == want
    rate = n / dt
    # the rate is reported, not gated: it depends on the host's Python threads and ctypes, not on parity
    print("\nqueue: %d n=1 Verify calls from 64 threads in %.3f s = %.0f Verify/s, %d batches" % (n, dt, rate, b1 - b0))
    assert b1 - b0 < n // 64, (b1 - b0, n)  # coalesced: far fewer launches than calls


# ---------------------------------------------------------------- cross-stream workspace ordering
def test_rlc_device_calls_on_two_streams(impl):
    """Two *_device RLC calls with different messages issued back to back on two streams share the H(m)
    table and fallback workspaces; each bitmap must still equal its own per-item Verify."""
    import ctypes
    import torch
    from charon_amd.tbls import load_library
    lib = load_library()
    dev = torch.device("cuda", 0)
    batches = []
    for seed in (10, 11):
        pks, msgs, sigs = _mixed_items(impl, 2048, seed)
        want = impl.batch_verify_status(pks, msgs, sigs)
        table = list(dict.fromkeys(msgs))
        pos = {m: j for j, m in enumerate(table)}
        batches.append(dict(
            pk=torch.frombuffer(bytearray(b"".join(pks)), dtype=torch.uint8).to(dev),
            sig=torch.frombuffer(bytearray(b"".join(sigs)), dtype=torch.uint8).to(dev),
            midx=torch.tensor([pos[m] for m in msgs], dtype=torch.int32).to(dev),
            msg=torch.frombuffer(bytearray(b"".join(table)), dtype=torch.uint8).to(dev),
            off=torch.arange(0, 32 * (len(table) + 1), 32, dtype=torch.int64).to(dev),
            st=torch.full((len(pks),), -7, dtype=torch.int32, device=dev), n=len(pks), nm=len(table), want=want))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for rep in range(3):
        for b, s in zip(batches, streams):
            b["st"].fill_(-7)
        torch.cuda.synchronize(dev)
        for b, s in zip(batches, streams):
            rc = lib.hipbls_batch_verify_rlc_device(b["pk"].data_ptr(), b["sig"].data_ptr(), b["midx"].data_ptr(),
                                                    b["n"], b["msg"].data_ptr(), b["off"].data_ptr(), b["nm"],
                                                    os.urandom(32), b["st"].data_ptr(), ctypes.c_void_p(s.cuda_stream))
            assert rc == 0
        torch.cuda.synchronize(dev)
        for b in batches:
            assert b["st"].cpu().tolist() == b["want"]


# ---------------------------------------------------------------- resident H(m) cache (§8f.2)
def test_hcache_hits_across_calls_same_statuses(impl):
    """The t partials of a validator arrive in separate calls (one parsigex message per peer): the second
    and later calls find every root in the cache; statuses are unchanged; eviction keeps results exact."""
    rng = random.Random(99)
    sks, pks = _keys(impl, rng, 64)
    roots = [rng.randbytes(32) for _ in range(48)]
    impl.hcache_config(64)
    try:
        calls = []
        for peer in range(4):  # each "peer" sends one partial per validator over the same roots
            sel = [(v * 4 + peer) % 64 for v in range(48)]
            sigs, _ = impl.sign_batch([sks[k] for k in sel], roots)
            sigs = list(sigs)
            if peer == 2:
                sigs[5] = sigs[6]
            calls.append(([pks[k] for k in sel], list(roots), sigs))
        h0 = impl.hcache_stats()
        for i, (p, m, s) in enumerate(calls):
            want = impl.batch_verify_status(p, m, s)
            assert impl.batch_verify_rlc_status(p, m, s) == want
        hits, misses, entries = impl.hcache_stats()
        assert misses - h0[1] == 48 and hits - h0[0] == 3 * 48 and entries == 48
        # a call with 40 new roots evicts most of the old ones: still exact
        new_roots = [rng.randbytes(32) for _ in range(40)]
        sigs, _ = impl.sign_batch(sks[:40], new_roots)
        mixed_m = new_roots + roots[:8]
        mixed_s = list(sigs) + list(calls[0][2][:8])
        mixed_p = pks[:40] + calls[0][0][:8]
        assert impl.batch_verify_rlc_status(mixed_p, mixed_m, mixed_s) == impl.batch_verify_status(mixed_p, mixed_m,
                                                                                                    mixed_s)
        assert impl.batch_verify_rlc_status(calls[1][0], calls[1][1], calls[1][2]) == [0] * 48
    finally:
        impl.hcache_config(0)


# ---------------------------------------------------------------- signing root on the GPU (§8f.3)
def test_verify_signed_data_signing_root_on_gpu(impl):
    from charon_amd.tbls import ERR_ZERO_SIG
    from oracle import ssz
    rng = random.Random(31)
    sks, pks = _keys(impl, rng, 8)
    objs = [rng.randbytes(32) for _ in range(8)]
    domain = ssz.compute_domain(bytes.fromhex("01000000"), bytes.fromhex("00001020"))  # DOMAIN_BEACON_ATTESTER
    roots = [ssz.signing_data_root(o, domain) for o in objs]
    sigs, _ = impl.sign_batch(sks, roots)
    sigs = list(sigs)
    sigs[3] = bytes(96)  # all-zero signature: eth2util/signing rejects it before tbls.Verify
    objs_v = list(objs)
    objs_v[5] = objs[6]
    got = impl.verify_signed_data_status(pks, objs_v, [domain] * 8, sigs)
    assert got == [0, 0, 0, ERR_ZERO_SIG, 0, 3, 0, 0]
    assert [g for i, g in enumerate(got) if i != 3] == [s for i, s in enumerate(
        impl.batch_verify_status(pks, [ssz.signing_data_root(o, domain) for o in objs_v], sigs)) if i != 3]


# ---------------------------------------------------------------- cluster-lock bulk verification (§8f.4)
def test_cluster_locks_bulk_verify(impl, kat):
    """Lock.VerifySignatures (cluster/lock.go:144-274) for all four example locks as ONE batched
    FastAggregateVerify launch, plus lock-003's threshold-aggregated builder registrations as one batch."""
    from oracle import ssz
    groups = []
    for lock in kat["locks"]:
        pks = [h(s) for v in lock["validators"] for s in v["public_shares"]]
        groups.append((pks, h(lock["signature_aggregate"]), h(lock["lock_hash"])))
    assert impl.batch_verify_aggregate_status(groups) == [0, 0, 0, 0]
    tampered = [(g[0], g[1], g[2][::-1]) for g in groups]
    assert impl.batch_verify_aggregate_status(groups + tampered) == [0] * 4 + [3] * 4
    lock = kat["locks"][3]
    domain = ssz.compute_domain(ssz.DOMAIN_APPLICATION_BUILDER, h(lock["fork_version"]))
    pks, objs, sigs = [], [], []
    for v in lock["validators"]:
        br = v["builder_registration"]
        objs.append(ssz.validator_registration_root(h(br["fee_recipient"]), br["gas_limit"], br["timestamp"],
                                                    h(br["pubkey"])))
        pks.append(h(v["distributed_public_key"]))
        sigs.append(h(br["signature"]))
    assert impl.verify_signed_data_status(pks, objs, [domain] * len(pks), sigs) == [0] * len(pks)


# ---------------------------------------------------------------- sigagg in one call (sigagg.go:138-159)
@pytest.mark.parametrize("layout", ["auto", "quads"])
def test_threshold_aggregate_verify_fused_equals_two_calls(impl, layout):
    """hipbls_threshold_aggregate_verify_batch == batch_threshold_aggregate + batch_verify_status of the
    aggregates, on honest groups, a failing aggregation (id 0, bad partial), a wrong root key, a wrong message,
    an identity root key and an all-infinity group (aggregate at infinity)."""
    from oracle import bls12381 as bls
    rng = random.Random(404)
    groups, dvpks, msgs = [], [], []
    secrets_ = []
    for g in range(40):
        secret = rng.randrange(1, R_ORDER)
        tail = [rng.randrange(R_ORDER) for _ in range(2)]
        ids = rng.sample(range(1, 9), 3)
        if g in (11, 12):  # ids off the small-integer Lagrange path (ops.h lagrange_small): L = 1, S = sigma
            ids = [2 ** 40 + 3 + g, 5, 2 ** 21]
        sh = _shares_at(secret, tail, ids)
        root = rng.randbytes(32)
        sigs, _ = impl.sign_batch([sh[i] for i in ids], [root] * 3)
        groups.append(dict(zip(ids, sigs)))
        secrets_.append(secret)
        msgs.append(root)
    dvpks, _ = impl.secret_to_public_key_batch([s.to_bytes(32, "big") for s in secrets_])
    dvpks = list(dvpks)
    groups[3] = {0: list(groups[3].values())[0], 5: list(groups[3].values())[1]}       # id 0: cannot combine
    k4 = list(groups[4])[0]
    bad = bytearray(groups[4][k4])
    bad[0] &= 0x7F
    groups[4] = dict(groups[4])
    groups[4][k4] = bytes(bad)                                                          # undecodable partial
    dvpks[5] = dvpks[6]                                                                 # wrong root key
    msgs[7] = rng.randbytes(32)                                                         # wrong message
    dvpks[8] = b"\xc0" + bytes(47)                                                      # identity key
    groups[9] = {1: b"\xc0" + bytes(95), 2: b"\xc0" + bytes(95)}                       # aggregate = infinity
    bad_pk = bytearray(dvpks[10])
    bad_pk[0] &= 0x7F
    dvpks[10] = bytes(bad_pk)                                                           # undecodable root key
    from charon_amd.tbls import PAIR_AUTO, PAIR_QUADS
    prev = impl.set_pair_mode(PAIR_QUADS if layout == "quads" else PAIR_AUTO)
    try:
        res, vst = impl.batch_threshold_aggregate_verify(groups, dvpks, msgs)
    finally:
        impl.set_pair_mode(prev)
    want_res = impl.batch_threshold_aggregate(groups)
    assert [r if isinstance(r, bytes) else str(r) for r in res] == \
        [r if isinstance(r, bytes) else str(r) for r in want_res]
    ok = [g for g, r in enumerate(want_res) if isinstance(r, bytes)]
    want_v = impl.batch_verify_status([dvpks[g] for g in ok], [msgs[g] for g in ok], [want_res[g] for g in ok])
    assert [vst[g] for g in ok] == want_v
    assert vst[3] == 5 and vst[4] == 2  # aggregation statuses carried over
    assert vst[5] == 3 and vst[7] == 3 and vst[8] == 3 and vst[9] == 3 and vst[10] == 1
    assert vst[11] == 0 and vst[12] == 0
    assert res[11] == bls.threshold_aggregate(groups[11])
    assert sum(1 for v in vst if v == 0) == 40 - 7
