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
