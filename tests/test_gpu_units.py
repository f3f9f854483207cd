"""Device builds of single pairing building blocks vs the host build and the oracle (ADVICE r02, lg2.h:263).

tests/native/libgpu_units.so runs the product's own device functions on the GPU:

* `final_exponentiation` (pairing.h), one lane per element, and `final_exponentiation_split` (lg2.h), a lane pair
  per element with DPP exchanges: equal to each other and to the host build on random elements; exactly 1 on the
  identity and on Fp2 elements.  The latter two make every saved compressed power degenerate (z2 = z3 = 0), so the
  lane-pair Karabina exponentiation takes its Granger-Scott fallback (`fp2_is_zero(pre[5])` -> fp12h_exp_xabs) on
  the device.
* `fp12h_exp_xabs_karabina` and `fp12h_exp_xabs` on split cyclotomic elements == the oracle's a^|x|, the identity
  included (the fallback again, with the result checked against the power itself).
"""
import ctypes
import random

import pytest

from oracle import bls12381 as bls
from tests.test_host_arith import f12_bytes, f12_from, rand_f12

pytestmark = pytest.mark.gpu

X_ABS = 0xD201000000010000


@pytest.fixture(scope="module")
def G():
    from tests.hostlib import gpu_units_lib
    return gpu_units_lib()


def _run(fn, elems, *extra):
    n = len(elems)
    inp = b"".join(f12_bytes(e) for e in elems)
    out = ctypes.create_string_buffer(576 * n)
    assert fn(inp, out, ctypes.c_uint64(n), *extra) == 0
    raw = out.raw
    return [f12_from(raw[576 * i:576 * i + 576]) for i in range(n)]


def _cyclotomic(rng):
    a = rand_f12(rng)
    c = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    return bls.f12_mul(bls.f12_pow(c, bls.P * bls.P), c)


def test_final_exponentiation_split_vs_one_lane_vs_host(G):
    from tests.hostlib import buf, lib
    L = lib()
    rng = random.Random(41)
    one = bls.F12_ONE
    z = (0, 0)
    fp2s = [(((rng.randrange(bls.P), rng.randrange(bls.P)), z, z), (z, z, z)) for _ in range(3)]
    rands = [rand_f12(rng) for _ in range(5)]
    elems = [one] + fp2s + rands
    a = _run(G.gu_final_exp, elems)
    b = _run(G.gu_final_exp_split, elems)
    assert a == b
    for e, got in zip(elems[:4], a[:4]):
        assert got == one
    out = buf(576)
    for e, got in zip(rands, a[4:]):
        L.ht_final_exp(f12_bytes(e), out)
        assert f12_from(out.raw) == got


@pytest.mark.parametrize("karabina", [1, 0])
def test_exp_xabs_split_vs_oracle(G, karabina):
    rng = random.Random(43 + karabina)
    elems = [bls.F12_ONE] + [_cyclotomic(rng) for _ in range(3)]
    got = _run(G.gu_exp_xabs_split, elems, ctypes.c_int(karabina))
    for e, g in zip(elems, got):
        assert g == bls.f12_pow(e, X_ABS)


@pytest.mark.parametrize("op", [0, 1])
def test_quad_final_exp_and_exp_xabs(G, op):
    """lg2.h final_exponentiation_quad (op 0) and fp12q_exp_xabs_karabina (op 1) on a lane quad: all four lanes agree,
    and equal the one-lane final exponentiation / the oracle's a^|x|; the identity and Fp2 elements take the
    quad's degenerate branch."""
    rng = random.Random(47 + op)
    z = (0, 0)
    fp2s = [(((rng.randrange(bls.P), rng.randrange(bls.P)), z, z), (z, z, z)) for _ in range(2)]
    if op == 0:
        elems = [bls.F12_ONE] + fp2s + [rand_f12(rng) for _ in range(4)]
        want = _run(G.gu_final_exp, elems)
    else:
        elems = [bls.F12_ONE] + [_cyclotomic(rng) for _ in range(4)]
        want = [bls.f12_pow(e, X_ABS) for e in elems]
    n = len(elems)
    inp = b"".join(f12_bytes(e) for e in elems)
    out = ctypes.create_string_buffer(4 * 576 * n)
    assert G.gu_quad(inp, out, ctypes.c_uint64(n), ctypes.c_int(op)) == 0
    raw = out.raw
    for i in range(n):
        lanes = [f12_from(raw[576 * (4 * i + q):576 * (4 * i + q) + 576]) for q in range(4)]
        assert lanes[0] == lanes[1] == lanes[2] == lanes[3] == want[i], i
