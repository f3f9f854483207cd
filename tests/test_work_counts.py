"""The roofline's algorithmic unit (bench.py FPMUL_PER_VERIFY) is the mean Fp-multiplication count
(fp_mul + fp_sqr, 381-bit Montgomery products) of one tbls.Verify of a C2 item, counted by the
instrumented host build of the same per-lane code the kernels run (tests/native/host_ops.cpp).
This test recomputes it on a seeded sample and keeps bench.py honest."""
import ctypes
import os
import random

from oracle import bls12381 as bls
from tests.hostlib import lib


def mean_verify_count(n=48, seed=0x636861726F6E):
    L = lib()
    rng = random.Random(seed)
    c = (ctypes.c_uint64 * 2)()
    tot = 0
    for _ in range(n):
        sk = rng.randrange(1, bls.R).to_bytes(32, "big")
        m = rng.randbytes(32)
        pk, s = bls.secret_to_public_key(sk), bls.sign(sk, m)
        L.ht_count_verify(pk, m, 32, s, c)
        tot += c[0] + c[1]
    return tot / n


def test_bench_fpmul_per_verify_matches_count():
    import bench
    got = mean_verify_count()
    assert abs(got - bench.FPMUL_PER_VERIFY) / got < 0.01, got


def test_bench_rlc_stage_counts_match():
    """bench.RLC_FPMUL (the RLC roofline's unit) against the host build of the four stages."""
    import bench
    from tests.rlc_cases import message_table, validator_batch
    from tests.test_rlc_host import host_pk, host_sign
    L = lib()

    def run(pks, msgs, sigs):
        table, idx = message_table(msgs)
        n = len(pks)
        offs = (ctypes.c_uint64 * (len(table) + 1))(*[32 * i for i in range(len(table) + 1)])
        st = (ctypes.c_int32 * n)()
        stats = (ctypes.c_uint64 * 3)()
        cnt = (ctypes.c_uint64 * 4)()
        arr = (ctypes.c_uint32 * n)(*idx)
        L.ht_rlc_verify(b"".join(pks), b"".join(sigs), arr, ctypes.c_uint64(n), b"".join(table), offs,
                        ctypes.c_uint64(len(table)), bytes(32), st, stats, cnt)
        return list(stats), list(cnt)

    want = bench.RLC_FPMUL
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 4, 4, seed=1)
    stats, cnt = run(pks, msgs, sigs)
    assert abs(cnt[0] / 16 - want["item"]) / want["item"] < 0.02
    assert abs(cnt[2] / 2 - want["window_2msg"]) / want["window_2msg"] < 0.02
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 1, 16, seed=2)
    stats, cnt = run(pks, msgs, sigs)
    assert abs(cnt[2] / 2 - want["window_1msg"]) / want["window_1msg"] < 0.02
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 4, 4, seed=3, bad=(1, 9))
    stats, cnt = run(pks, msgs, sigs)
    assert abs(cnt[3] / stats[2] - want["fallback"]) / want["fallback"] < 0.03


def test_bench_rlcb_stage_counts_match():
    """bench.RLCB_FPMUL (the batch-wide check's unit) against the host build of its stages."""
    import bench
    from tests.rlc_cases import message_table, validator_batch
    from tests.test_rlc_host import host_pk, host_sign
    L = lib()
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 16, 4, seed=5)  # 64 items, 4 chunks of 4 runs
    table, idx = message_table(msgs)
    n = len(pks)
    offs = (ctypes.c_uint64 * (len(table) + 1))(*[32 * i for i in range(len(table) + 1)])
    st = (ctypes.c_int32 * n)()
    passed = ctypes.c_int32()
    cnt = (ctypes.c_uint64 * 6)()
    arr = (ctypes.c_uint32 * n)(*idx)
    L.ht_rlcb_verify(b"".join(pks), b"".join(sigs), arr, ctypes.c_uint64(n), b"".join(table), offs,
                     ctypes.c_uint64(len(table)), bytes(32), st, ctypes.byref(passed), cnt)
    assert passed.value == 1 and cnt[5] == 0  # decided by the batch-wide check alone
    want = bench.RLCB_FPMUL
    assert abs(cnt[0] / n - want["item"]) / want["item"] < 0.02
    assert abs(cnt[3] / 4 - want["chunk_4runs"]) / want["chunk_4runs"] < 0.02
    # committee roots: 16 items of one root per chunk, one run (C4(ii))
    pks, msgs, sigs, _ = validator_batch(host_sign(L), host_pk(L), 4, 16, seed=6)
    table, idx = message_table(msgs)
    offs = (ctypes.c_uint64 * (len(table) + 1))(*[32 * i for i in range(len(table) + 1)])
    arr = (ctypes.c_uint32 * len(pks))(*idx)
    st = (ctypes.c_int32 * len(pks))()
    L.ht_rlcb_verify(b"".join(pks), b"".join(sigs), arr, ctypes.c_uint64(len(pks)), b"".join(table), offs,
                     ctypes.c_uint64(len(table)), bytes(32), st, ctypes.byref(passed), cnt)
    assert passed.value == 1
    assert abs(cnt[3] / 4 - want["chunk_1run"]) / want["chunk_1run"] < 0.02


def test_bench_rlcb_g1_counts_match():
    """bench.RLCB_FPMUL's G1 MSM units (g1msm.h) at one committee root of 512 partials, as C4(ii): stage 1 without
    the per-item Shamir multiplication, the G1 bucket + fold work per item (MSM stage with minus without the G1 MSM:
    the G2 MSM is the same in both), one Miller pair for the root."""
    import bench
    from tests.test_rlcb_host import _with_g1_min, committee_batch, rlcb
    L = lib()
    pks, msgs, sigs = committee_batch(L, [512], seed=41)
    on, off = (ctypes.c_uint64 * 6)(), (ctypes.c_uint64 * 6)()
    assert _with_g1_min(L, 64, lambda: rlcb(L, pks, msgs, sigs, counts=on)) == ([0] * 512, 1)
    assert _with_g1_min(L, 0, lambda: rlcb(L, pks, msgs, sigs, counts=off)) == ([0] * 512, 1)
    want = bench.RLCB_FPMUL
    assert abs(on[0] / 512 - want["item_g1slot"]) / want["item_g1slot"] < 0.02
    assert abs(off[0] / 512 - want["item"]) / want["item"] < 0.02
    assert abs((on[2] - off[2]) / 512 - want["g1msm_per_item_512"]) / want["g1msm_per_item_512"] < 0.03
    assert abs(on[3] - want["g1miller_per_root"]) / want["g1miller_per_root"] < 0.02


def test_bench_tagg_counts_match():
    """bench.TAGG_FPMUL (the C3 roofline's per-aggregate unit) against the host build of the fused sigagg stages over
    seeded 7-of-10 groups on ids 1..10 (the small-integer Lagrange path the bench's groups take)."""
    import bench
    L = lib()
    rng = random.Random(0xC3)
    tot = [0] * 5
    N = 4
    for _ in range(N):
        secret = rng.randrange(1, bls.R)
        poly = [secret] + [rng.randrange(bls.R) for _ in range(6)]
        ids = sorted(rng.sample(range(1, 11), 7))
        msg = rng.randbytes(32)
        sigs = []
        for i in ids:
            acc = 0
            for c in reversed(poly):
                acc = (acc * i + c) % bls.R
            sigs.append(bls.sign(acc.to_bytes(32, "big"), msg))
        pk = bls.secret_to_public_key(secret.to_bytes(32, "big"))
        out = (ctypes.c_uint64 * 5)()
        assert L.ht_count_tagg_verify(b"".join(sigs), (ctypes.c_int64 * 7)(*ids), 7, pk, msg, 32, out) == 0
        tot = [a + b for a, b in zip(tot, out)]
    want = bench.TAGG_FPMUL
    for k, got in zip(("scale_7", "sum", "unscale", "key_prep", "pairing"), tot):
        assert abs(got / N - want[k]) / want[k] < 0.03, (k, got / N)


def test_bench_auto_period_matches_library():
    """bench.RLC_AUTO_PERIOD = the library's back-off after a failed batch-wide check + the retried call."""
    import re
    import bench
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "charon_amd", "csrc",
                            "hipbls.hip")).read()
    backoff = int(re.search(r"constexpr int kRlcbBackoff = (\d+);", src).group(1))
    assert bench.RLC_AUTO_PERIOD == backoff + 1
