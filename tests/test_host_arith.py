"""Layer-by-layer parity of the kernel arithmetic (host build, tests/native) against the oracle.

The kernels' per-lane code in charon_amd/csrc is compiled for x86 here, so every field/tower/curve/
hash/pairing layer is diffed against oracle/bls12381.py on the CPU.  The GPU tests then only have to
show the device build computes the same thing (tests/test_gpu_parity.py).
"""
import random

import pytest

from oracle import bls12381 as bls
from tests.hostlib import buf, lib

P = bls.P


def be48(v):
    return v.to_bytes(48, "big")


def fp_from(b):
    return int.from_bytes(b, "big")


def g1_bytes(pt):
    return be48(pt[0]) + be48(pt[1])


def g2_bytes(pt):
    (x0, x1), (y0, y1) = pt
    return be48(x0) + be48(x1) + be48(y0) + be48(y1)


def g2_from(b):
    v = [fp_from(b[48 * i:48 * i + 48]) for i in range(4)]
    return ((v[0], v[1]), (v[2], v[3]))


def f12_from(b):
    c = [fp_from(b[48 * i:48 * i + 48]) for i in range(12)]
    f2 = [(c[2 * i], c[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def f12_bytes(f):
    out = b""
    for f6 in f:
        for f2 in f6:
            out += be48(f2[0]) + be48(f2[1])
    return out


def rand_f12(rng):
    return tuple(tuple((rng.randrange(P), rng.randrange(P)) for _ in range(3)) for _ in range(2))


@pytest.fixture(scope="module")
def L():
    return lib()


def test_expand_message(L):
    out = buf(256)
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    for msg in [b"", b"abc", b"a" * 200]:
        L.ht_expand_message(msg, len(msg), dst, len(dst), out)
        assert out.raw == bls.expand_message_xmd(msg, dst, 256)
    # 32-byte messages with a 43-byte DST take the word-assembled form (h2c.h expand_message_xmd_256_m32_d43): the
    # POP suite's DST and another 43-byte one (the DST bytes are read, not assumed)
    rng = random.Random(11)
    pop = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    assert len(pop) == 43
    for d in (pop, bytes(rng.randrange(256) for _ in range(43))):
        for msg in [bytes(32), b"\xff" * 32] + [bytes(rng.randrange(256) for _ in range(32)) for _ in range(6)]:
            L.ht_expand_message(msg, 32, d, 43, out)
            assert out.raw == bls.expand_message_xmd(msg, d, 256)


def test_map_to_curve(L):
    """Both SSWU candidates (gx1 square / not: the shared-exponentiation path of h2c.h) and the exceptional
    u = 0 (tv1 = 0, x1 = B/(ZA)), against the oracle's straight RFC 9380 map."""
    rng = random.Random(7)
    out = buf(192)
    branches = set()
    for u in [(0, 0), (1, 0), (0, 1)] + [(rng.randrange(P), rng.randrange(P)) for _ in range(16)]:
        L.ht_map_to_curve(be48(u[0]) + be48(u[1]), out)
        assert g2_from(out.raw) == bls.map_to_curve_sswu(u), u
        # which candidate the RFC picks: x1 = -B/A (1 + 1/(Z^2 u^4 + Z u^2)) (or B/(ZA)), gx1 square?
        zu2 = bls.f2_mul(bls.SSWU_Z, bls.f2_sqr(u))
        den = bls.f2_add(bls.f2_sqr(zu2), zu2)
        if bls.f2_is_zero(den):
            x1 = bls.f2_mul(bls.SSWU_B, bls.f2_inv(bls.f2_mul(bls.SSWU_Z, bls.SSWU_A)))
        else:
            x1 = bls.f2_mul(bls.f2_mul(bls.f2_neg(bls.SSWU_B), bls.f2_inv(bls.SSWU_A)),
                            bls.f2_add((1, 0), bls.f2_inv(den)))
        gx1 = bls.f2_add(bls.f2_add(bls.f2_mul(bls.f2_sqr(x1), x1), bls.f2_mul(bls.SSWU_A, x1)), bls.SSWU_B)
        branches.add(bls.f2_is_square(gx1))
    assert branches == {True, False}


def test_hash_to_g2(L):
    out = buf(192)
    for msg, dst in [(b"", b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"),
                     (b"abc", b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"),
                     (b"hello obol!", bls.DST_POP), (bytes(range(32)), bls.DST_POP)]:
        L.ht_hash_to_g2(msg, len(msg), dst, len(dst), out)
        assert g2_from(out.raw) == bls.hash_to_g2(msg, dst)


def test_clear_cofactor_matches_h_eff(L):
    rng = random.Random(3)
    out = buf(192)
    for _ in range(3):
        pt = bls.iso_map_g2(bls.map_to_curve_sswu((rng.randrange(P), rng.randrange(P))))
        L.ht_g2_clear_cofactor(g2_bytes(pt), out)
        assert g2_from(out.raw) == bls.g2_mul(pt, bls.H_EFF_G2)


def _random_g1_point(rng):
    while True:
        x = rng.randrange(P)
        y = bls.fp_sqrt((x ** 3 + 4) % P)
        if y is not None:
            return (x, y)


def _random_g2_point(rng):
    while True:
        x = (rng.randrange(P), rng.randrange(P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            return (x, y)


def test_g1_subgroup_check_vs_order(L):
    rng = random.Random(11)
    for _ in range(4):
        pt = _random_g1_point(rng)  # almost surely not in G1
        assert L.ht_g1_in_subgroup(g1_bytes(pt)) == int(bls.g1_mul(pt, bls.R) is None)
        pt_in = bls.g1_mul(pt, 0x396C8C005555E1568C00AAAB0000AAAB)  # cofactor h1 -> lands in G1
        assert L.ht_g1_in_subgroup(g1_bytes(pt_in)) == 1


def test_g2_subgroup_check_vs_order(L):
    rng = random.Random(12)
    for _ in range(3):
        pt = _random_g2_point(rng)
        assert L.ht_g2_in_subgroup(g2_bytes(pt)) == int(bls.g2_mul(pt, bls.R) is None) == 0
        pt_in = bls.g2_mul(pt, bls.H_EFF_G2)
        assert L.ht_g2_in_subgroup(g2_bytes(pt_in)) == 1


def test_g2_subgroup_and_small_multiple_one_chain(L):
    """ops.h g2_subgroup_and_mul_i64 (k_tagg_scale, small Lagrange integers): the membership answer equals the
    order test's and [c] P equals the oracle's, for points in and out of G2, signed c, c = +-1 and c past |x|'s
    top bit."""
    import ctypes
    rng = random.Random(21)
    out, inf = buf(192), ctypes.c_int(0)
    fn = L.ht_g2_subgroup_and_mul_i64
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    for trial in range(3):
        pt = _random_g2_point(rng)
        pt_in = bls.g2_mul(pt, bls.H_EFF_G2)
        for p, member in [(pt, 0), (pt_in, 1)]:
            for c in [1, -1, 5, -36, rng.randrange(1, 1 << 40), -rng.randrange(1, 1 << 62), (1 << 63) - 1]:
                assert fn(g2_bytes(p), c, out, ctypes.byref(inf)) == member
                want = bls.g2_mul(p, c) if c > 0 else bls.g2_neg(bls.g2_mul(p, -c))
                assert inf.value == int(want is None)
                if want is not None:
                    assert g2_from(out.raw) == want, (trial, member, c)


def test_decompress_roundtrip(L):
    rng = random.Random(5)
    out1, out2 = buf(96), buf(192)
    for _ in range(3):
        k = rng.randrange(1, bls.R)
        p1 = bls.g1_mul(bls.G1_GEN, k)
        assert L.ht_g1_decompress(bls.g1_compress(p1), 1, out1) == 0
        assert out1.raw == g1_bytes(p1)
        p2 = bls.g2_mul(bls.G2_GEN, k)
        assert L.ht_g2_decompress(bls.g2_compress(p2), 1, out2) == 0
        assert g2_from(out2.raw) == p2


def test_fp12_ops(L):
    rng = random.Random(9)
    out = buf(576)
    a, b = rand_f12(rng), rand_f12(rng)
    L.ht_fp12_op(0, f12_bytes(a), f12_bytes(b), out)
    assert f12_from(out.raw) == bls.f12_mul(a, b)
    L.ht_fp12_op(1, f12_bytes(a), f12_bytes(b), out)
    assert f12_from(out.raw) == bls.f12_mul(a, a)
    L.ht_fp12_op(2, f12_bytes(a), f12_bytes(b), out)
    assert f12_from(out.raw) == bls.f12_inv(a)
    for op, j in ((3, 1), (4, 2), (5, 3)):
        L.ht_fp12_op(op, f12_bytes(a), f12_bytes(b), out)
        assert f12_from(out.raw) == bls.f12_pow(a, P ** j)
    # cyclotomic squaring on an element of the cyclotomic subgroup: a^((p^6-1)(p^2+1))
    c = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
    c = bls.f12_mul(bls.f12_pow(c, P * P), c)
    L.ht_fp12_op(6, f12_bytes(c), f12_bytes(b), out)
    assert f12_from(out.raw) == bls.f12_mul(c, c)
    # sparse line multiplication vs dense
    z = (0, 0)
    line = ((b[0][0], b[0][1], z), (z, b[1][1], z))
    L.ht_fp12_op(7, f12_bytes(a), f12_bytes(line), out)
    assert f12_from(out.raw) == bls.f12_mul(a, line)


def test_pairing_matches_oracle_cubed(L):
    out = buf(576)
    k1, k2 = 0x1234567, 0x89ABCDEF
    P1 = bls.g1_mul(bls.G1_GEN, k1)
    Q1 = bls.g2_mul(bls.G2_GEN, k2)
    L.ht_pairing(g1_bytes(P1), g2_bytes(Q1), out)
    e = bls.pairing(P1, Q1)
    assert f12_from(out.raw) == bls.f12_mul(bls.f12_mul(e, e), e)


def test_sign_and_verify_kats(L, kat):
    k = kat["prysm"]
    out = buf(96)
    assert L.ht_sign(bytes.fromhex(k["sk"]), bytes.fromhex(k["signing_root"]), 32, out) == 0
    assert out.raw.hex() == k["sig"]
    pk = buf(48)
    assert L.ht_sk_to_pk(bytes.fromhex(k["sk"]), pk) == 0
    assert pk.raw == bls.secret_to_public_key(bytes.fromhex(k["sk"]))
    root = bytes.fromhex(k["signing_root"])
    assert L.ht_verify(pk.raw, root, 32, out.raw) == 0
    assert L.ht_verify(pk.raw, root[:-1] + b"\x00", 32, out.raw) == 3
    bad = bytearray(out.raw)
    bad[5] ^= 1
    assert L.ht_verify(pk.raw, root, 32, bytes(bad)) in (2, 3)
    assert L.ht_verify(bytes(48), root, 32, out.raw) == 1


def test_threshold_aggregate_host(L):
    msg = b"hello obol!"
    secret = 0xABCDEF0123456789
    shares = bls.threshold_split_poly(secret, [11, 22, 33], 7)
    ids = [2, 3, 5, 7]
    sigs = b"".join(bls.sign(shares[i], msg) for i in ids)
    import ctypes
    arr = (ctypes.c_int64 * 4)(*ids)
    out = buf(96)
    assert L.ht_threshold_aggregate(sigs, arr, 4, out) == 0
    assert out.raw == bls.sign(bls.sk_serialize(secret), msg)


def test_fixtures_verify_host(L):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")) as f:
        fx = json.load(f)
    for c in fx["verify"]:
        msg = bytes.fromhex(c["msg"])
        st = L.ht_verify(bytes.fromhex(c["pk"]), msg, len(msg), bytes.fromhex(c["sig"]))
        assert st == c["status"], c["note"]


def test_binary_gcd_inverse(L):
    """field.h fp_inv (Pornin's binary GCD, 27 x 30 divsteps) equals the Fermat power x^(p-2) and the oracle's
    inverse on Montgomery-form inputs: 0 (inverse 0), 1, p - 1, powers of two, near-p values, Fibonacci-like
    inputs (the slowest-converging GCD inputs) and random values."""
    import ctypes
    import random as _r
    P = bls.P
    R = 1 << 384
    rng = _r.Random(11)
    fib = [1, 1]
    while fib[-1] < P:
        fib.append(fib[-1] + fib[-2])
    xs = [0, 1, 2, P - 1, P - 2, (P - 1) // 2] + [(1 << k) % P for k in range(0, 381, 17)] + fib[-12:] + \
        [f % P for f in fib[-12:]] + [rng.randrange(P) for _ in range(300)]
    fn = L.ht_fp_inv
    for x in xs:
        x %= P
        xm = x * R % P  # Montgomery form of x
        inp = (ctypes.c_uint32 * 12)(*[(xm >> (32 * i)) & 0xFFFFFFFF for i in range(12)])
        outs = []
        for gcd in (1, 0):
            o = (ctypes.c_uint32 * 12)()
            fn(inp, gcd, o)
            outs.append(sum(v << (32 * i) for i, v in enumerate(o)))
        want = (pow(x, P - 2, P) * R) % P
        assert outs[0] == outs[1] == want, hex(x)
    # the divstep bound also covers non-canonical operands below 2^382 (p + 1, 2p - 1: 763 divsteps <= 27 x 30)
    for xm in (P, P + 1, 2 * P - 1, 2 * P - 2, (1 << 382) - 1):
        inp = (ctypes.c_uint32 * 12)(*[(xm >> (32 * i)) & 0xFFFFFFFF for i in range(12)])
        o = (ctypes.c_uint32 * 12)()
        fn(inp, 1, o)
        got = sum(v << (32 * i) for i, v in enumerate(o))
        x = xm * pow(R, -1, P) % P
        assert got == (pow(x, P - 2, P) * R) % P, hex(xm)


def test_compressed_cyclotomic_exponentiation(L):
    """a^|x| by Karabina's compressed squarings + batch decompression (pairing.h) == Granger-Scott == the oracle's
    power, on cyclotomic elements; the degenerate inputs (the identity, an Fp2 element's easy-part image) take the
    Granger-Scott fallback and still give the exact power; and final_exponentiation of 1 and of Fp2 elements is 1."""
    rng = random.Random(17)
    out = buf(576)
    X_ABS = 0xD201000000010000
    one = bls.F12_ONE
    cases = []
    for _ in range(3):
        a = rand_f12(rng)
        c = bls.f12_mul(bls.f12_conj(a), bls.f12_inv(a))
        cases.append(bls.f12_mul(bls.f12_pow(c, P * P), c))
    cases.append(one)
    for c in cases:
        want = bls.f12_pow(c, X_ABS)
        for op in (8, 9):
            L.ht_fp12_op(op, f12_bytes(c), f12_bytes(c), out)
            assert f12_from(out.raw) == want, op
    z = (0, 0)
    for f in (one, (((rng.randrange(P), rng.randrange(P)), z, z), (z, z, z))):
        L.ht_final_exp(f12_bytes(f), out)
        assert f12_from(out.raw) == one
        L.ht_final_exp_l(f12_bytes(f), out)  # the LDS-accumulator variant takes the same degenerate branch
        assert f12_from(out.raw) == one
    want, got = buf(576), buf(576)
    for _ in range(2):  # random elements: the LDS-accumulator final exponentiation equals the register one
        f = rand_f12(rng)
        L.ht_final_exp(f12_bytes(f), want)
        L.ht_final_exp_l(f12_bytes(f), got)
        assert got.raw == want.raw


def test_verify_signature_membership_from_miller_loop(L):
    """op_verify takes the signature's G2 membership from the Miller loop's [|x|] sig (pairing.h
    g2_subgroup_from_miller).  Statuses must equal the oracle's (herumi.go:285-301 order) for: honest and
    wrong-message signatures, a random curve point outside G2, small-order points (order 13 and 23: the loop's
    doubling/addition steps hit their exceptional cases, Z = 0), a small-order point times an honest signature,
    and the same signatures under an infinity public key (the early-exit path keeps the separate check)."""
    rng = random.Random(23)
    x = -bls.X_ABS
    h2 = (x ** 8 - 4 * x ** 7 + 5 * x ** 6 - 4 * x ** 4 + 6 * x ** 3 - 4 * x ** 2 - 4 * x + 13) // 9
    n2 = h2 * bls.R

    def random_point():
        while True:
            px = (rng.randrange(P), rng.randrange(P))
            py = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(px), px), bls.B2))
            if py is not None:
                return (px, py)

    def of_order(q):  # the q-part of a random point, reduced to order exactly q (q^2 divides the cofactor)
        m = n2
        while m % q == 0:
            m //= q
        while True:
            pt = bls.g2_mul(random_point(), m)
            if pt is None:
                continue
            while bls.g2_mul(pt, q) is not None:
                pt = bls.g2_mul(pt, q)
            return pt

    sk = rng.randrange(1, bls.R).to_bytes(32, "big")
    msg = rng.randbytes(32)
    pk = bls.secret_to_public_key(sk)
    sig = bls.sign(sk, msg)
    sig_pt = bls.g2_decompress(sig)
    sigs = [sig, bls.g2_compress(random_point())]
    for q in (13, 23):
        small = of_order(q)
        sigs.append(bls.g2_compress(small))
        sigs.append(bls.g2_compress(bls.g2_add(sig_pt, small)))
    inf_pk = bytes([0xC0]) + bytes(47)
    # the oracle's statuses (pinned on one case each; the rest follow herumi's order: a signature outside G2 fails
    # deserialization, status 2, before the infinity key or the pairing matter)
    assert bls.verify_status(pk, msg, sig) == 0 and bls.verify_status(inf_pk, msg, sigs[2]) == 2
    for k, s in enumerate(sigs):
        for p, m, want in ((pk, msg, 0 if k == 0 else 2), (pk, msg[::-1], 3 if k == 0 else 2),
                           (inf_pk, msg, 3 if k == 0 else 2)):
            assert L.ht_verify(p, m, 32, s) == want, (k, want)
            assert L.ht_verify_l(p, m, 32, s) == want, (k, want)  # k_verify_fused's LDS-resident Miller loop


def test_miller_loop_lds_resident_f_matches_registers(L):
    """pairing_lds.h miller_loop_2_l (k_verify_fused: f in LDS, squaring and line products reordered in place) returns
    the same f and the same final T as pairing.h miller_loop_2 (pinned to the oracle through ht_verify and the fixture
    tests), limb for limb, for Verify-shaped operands: a G1 key, H(m), -g1 and a signature in or outside G2."""
    rng = random.Random(29)
    f_reg, f_lds, t_reg, t_lds = buf(576), buf(576), buf(288), buf(288)
    neg_g1 = (bls.G1_GEN[0], (-bls.G1_GEN[1]) % P)
    for trial in range(3):
        p0 = bls.g1_mul(bls.G1_GEN, rng.randrange(1, bls.R))
        q0 = bls.hash_to_g2(rng.randbytes(32), bls.DST_POP)
        q1 = bls.g2_mul(q0, rng.randrange(1, bls.R)) if trial else _random_g2_point(rng)
        args = (g1_bytes(p0), g2_bytes(q0), g1_bytes(neg_g1), g2_bytes(q1))
        L.ht_miller2(*args, 0, f_reg, t_reg)
        L.ht_miller2(*args, 1, f_lds, t_lds)
        assert f_lds.raw == f_reg.raw and t_lds.raw == t_reg.raw, trial


def test_lagrange_small_integers(L):
    """ops.h lagrange_small: for small share ids, c_k = N_k (L / D_k) is an exact integer with c_k = lambda_k L mod r
    (so sum lambda_k sig_k = [L^-1] sum c_k sig_k); large, zero or duplicate ids take the field path (0)."""
    import ctypes
    R = bls.R
    rng = random.Random(9)
    cases = [[1, 2, 3], list(range(1, 11))[:7], [3, 7, 1, 10, 2, 9, 5], [-3, 5, 2], list(range(1, 17)),
             [1, 1 << 20], [5]]
    for _ in range(20):
        n = rng.randrange(2, 11)
        cases.append(rng.sample(range(1, 40), n))
    from math import gcd, prod

    def expect(ids):  # the exact integers, and whether all of them fit the 63-bit path
        t = len(ids)
        D = [prod(ids[j] - ids[k] for j in range(t) if j != k) for k in range(t)]
        Lx = 1
        for d in D:
            Lx = Lx * abs(d) // gcd(Lx, abs(d))
        N = [prod(ids[j] for j in range(t) if j != k) for k in range(t)]
        c = [N[k] * (Lx // abs(D[k])) * (1 if D[k] > 0 else -1) for k in range(t)]
        fits = t <= 16 and all(abs(v) < 2 ** 63 for v in D + N + c + [Lx])
        return fits, c, Lx

    n_small = 0
    for ids in cases:
        t = len(ids)
        arr = (ctypes.c_int64 * t)(*ids)
        lam = bls.lagrange_coeffs_at_zero(ids)
        fits, cx, Lx = expect(ids)
        n_small += fits
        for me in range(t):
            c, Lv = ctypes.c_int64(), ctypes.c_uint64()
            ok = L.ht_lagrange_small(arr, t, me, ctypes.byref(c), ctypes.byref(Lv))
            assert ok == int(fits), ids
            if ok:
                assert c.value == cx[me] and Lv.value == Lx
                assert (c.value - lam[me] * Lv.value) % R == 0, (ids, me)
    assert n_small >= 20
    for ids in ([1, 2, 1 << 21], [0, 1, 2], [4, 4, 1], [1 << 40, 3], list(range(1, 18))):
        arr = (ctypes.c_int64 * len(ids))(*ids)
        c, Lv = ctypes.c_int64(), ctypes.c_uint64()
        assert L.ht_lagrange_small(arr, len(ids), 0, ctypes.byref(c), ctypes.byref(Lv)) == 0, ids
