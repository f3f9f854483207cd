"""4-dimensional GLS scalar multiplication on G2 (curve.h g2_mul_glv4), used by ThresholdAggregate's
lambda_k * sigma_k (k_tagg_scale) and by Sign.  Host build of the kernel code: the split result
must equal plain double-and-add and the oracle's [k]P on subgroup points, for random scalars and
for the digit-boundary scalars of the base-|x| expansion."""
import ctypes
import random

import pytest

from oracle import bls12381 as bls
from tests.hostlib import buf, lib

X_ABS = 0xD201000000010000


@pytest.fixture(scope="module")
def L():
    return lib()


def _k8(k):
    return (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def _scalars(seed):
    rnd = random.Random(seed)
    edge = [0, 1, 2, X_ABS - 1, X_ABS, X_ABS + 1, X_ABS ** 2, X_ABS ** 3 - 1, X_ABS ** 3,
            bls.R - 1, bls.R - X_ABS, (bls.R - 1) // 2]
    return edge + [rnd.randrange(bls.R) for _ in range(12)] + [rnd.randrange(1 << 64) for _ in range(3)]


def test_glv4_matches_double_and_add_and_oracle(L):
    rnd = random.Random(11)
    pts = [bls.sign(rnd.randrange(1, bls.R).to_bytes(32, "big"), rnd.randbytes(32)) for _ in range(3)]
    for p96 in pts:
        for k in _scalars(rnd.randrange(1 << 30)):
            a, b = buf(96), buf(96)
            assert L.ht_g2_mul(p96, _k8(k), 1, a) == 0
            assert L.ht_g2_mul(p96, _k8(k), 0, b) == 0
            assert a.raw == b.raw, hex(k)
        k = rnd.randrange(bls.R)
        a = buf(96)
        L.ht_g2_mul(p96, _k8(k), 1, a)
        want = bls.g2_compress(bls.g2_mul(bls.g2_decompress(p96), k))
        assert a.raw == want
