"""The roofline's algorithmic unit (bench.py FPMUL_PER_VERIFY) is the mean Fp-multiplication count
(fp_mul + fp_sqr, 381-bit Montgomery products) of one tbls.Verify of a C2 item, counted by the
instrumented host build of the same per-lane code the kernels run (tests/native/host_ops.cpp).
This test recomputes it on a seeded sample and keeps bench.py honest."""
import ctypes
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
