"""CPU oracle: spec-literal restatement of the BLS12-381 arithmetic behind charon's tbls path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (charon_amd/, include/, the HIP library)
imports or links this file.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may use it, and only as the checker.

What it restates
----------------
charon's hot path (tbls.Verify / tbls.ThresholdAggregate) delegates all arithmetic to the
third-party module github.com/herumi/bls-eth-go-binary v1.32.1 (/root/reference/go.mod:14,
go.sum:297-298), which is NOT vendored in /root/reference.  Its algorithm is the published
Ethereum BLS scheme, which this module restates from the public standards:

* draft-irtf-cfrg-bls-signature (cited at /root/reference/tbls/tbls.go:62-67): minimal-pubkey-size
  variant, proof-of-possession ciphersuite  BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_
  (herumi EthModeLatest, selected at /root/reference/tbls/herumi.go:29-33);
* RFC 9380 hash_to_curve (expand_message_xmd/SHA-256, simplified SWU on the 3-isogenous curve,
  isogeny map, h_eff cofactor clearing);
* ZCash compressed point encoding (48-byte G1, 96-byte G2);
* optimal ate pairing (computed here with affine Miller steps over a generic Fp12 and a plain
  final exponentiation by (p^12-1)/r -- deliberately NOT the projective/sparse formulas the
  HIP engine uses, so the two are independent restatements).

Semantics follow /root/reference/tbls/herumi.go:
  Verify             herumi.go:285-301  (pk deserialize -> sig deserialize -> pairing check)
  ThresholdAggregate herumi.go:244-283  (Lagrange at 0 over Fr with 1-based decimal ids)
  Sign               herumi.go:303-313
  SecretToPublicKey  herumi.go:67-80    (GetSafePublicKey: zero secret is an error)
  Aggregate          herumi.go:220-242
  VerifyAggregate    herumi.go:315-339  (FastAggregateVerify)
  ThresholdSplit     herumi.go:134-181  (share_i = sum_j poly_j * i^j)
  RecoverSecret      herumi.go:183-218

Pinning: every herumi-produced vector in the reference (tests/golden/kat_reference.json, built by
tests/golden/make_kat_reference.py from the reference's own test files) is checked against this
module in tests/test_oracle_kat.py.  Edge semantics the reference does not pin (infinity keys,
non-canonical encodings, id 0 / duplicate ids) are chosen explicitly in `EDGE_POLICY` below.
"""

from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # BLS parameter x = -X_ABS
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

EDGE_POLICY = {
    "pk_infinity": "deserializes; Verify/VerifyAggregate fail (IETF KeyValidate)",
    "sig_infinity": "deserializes; pairing check decides (always fails for a valid pk)",
    "non_canonical_x": "x >= p is a deserialize error",
    "missing_compression_flag": "deserialize error (48/96-byte inputs must be compressed)",
    "infinity_with_payload": "0x40 flag with any other non-zero bit is a deserialize error",
    "not_on_curve / not_in_subgroup": "deserialize error",
    "recover_id_zero_or_duplicate": "error 'cannot combine signatures'",
    "recover_single_share": "returns that share's point re-serialized",
    "fast_aggregate_verify_empty": "fails",
    "aggregate_empty": "no error: the sum of nothing is the point at infinity, 0xc0 || 0^95 "
                       "(herumi.go:220-242 has no empty check; sig.Aggregate leaves the zero point)",
    "share_id": "a Go int parsed as Fr (strconv.Itoa -> SetDecString, herumi.go:264-271): id mod r, so "
                "-k is r - k; id = 0 and duplicate ids fail to combine",
    "secret_zero": "SecretToPublicKey error; secret >= r is a deserialize error",
}


class BLSError(Exception):
    """Error carrying the same message strings tbls.Herumi wraps (herumi.go)."""


# ----------------------------------------------------------------------------------------------
# Fp, Fp2
# ----------------------------------------------------------------------------------------------
def inv(a: int) -> int:
    return pow(a, -1, P)


def fp_sqrt(a: int) -> Optional[int]:
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a % P else None


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# Fp2 = Fp[u]/(u^2+1), element (c0, c1) = c0 + c1*u
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, k: int):
    return (a[0] * k % P, a[1] * k % P)


def f2_inv(a):
    n = inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_pow(a, e: int):
    res = F2_ONE
    base = a
    while e:
        if e & 1:
            res = f2_mul(res, base)
        base = f2_sqr(base)
        e >>= 1
    return res


def f2_is_zero(a) -> bool:
    return a[0] % P == 0 and a[1] % P == 0


def f2_is_square(a) -> bool:
    return fp_is_square((a[0] * a[0] + a[1] * a[1]) % P)


def f2_sqrt(a) -> Optional[Tuple[int, int]]:
    """Any square root of a in Fp2 (p = 3 mod 4); the caller fixes the sign."""
    if f2_is_zero(a):
        return F2_ZERO
    # complex method: a = a0 + a1 u, find x with x^2 = a
    a0, a1 = a[0] % P, a[1] % P
    n = fp_sqrt((a0 * a0 + a1 * a1) % P)
    if n is None:
        return None
    half = inv(2)
    for s in (n, (-n) % P):
        t = (a0 + s) * half % P
        x0 = fp_sqrt(t)
        if x0 is None:
            continue
        if x0 == 0:
            # then a1 must be 0 and a0 = -x1^2
            x1 = fp_sqrt((-a0) % P)
            if x1 is None:
                continue
            cand = (0, x1)
        else:
            cand = (x0, a1 * inv(2 * x0) % P)
        if f2_sqr(cand) == (a0, a1):
            return cand
    return None


def sgn0_fp2(a) -> int:
    """RFC 9380 sgn0 for m = 2."""
    s0 = a[0] % 2
    z0 = a[0] % P == 0
    s1 = a[1] % 2
    return s0 | (z0 & s1)


# ----------------------------------------------------------------------------------------------
# Fp12 as a tower Fp2[v]/(v^3 - xi), Fp6[w]/(w^2 - v), xi = 1 + u.  Generic (dense) arithmetic only.
# ----------------------------------------------------------------------------------------------
XI = (1, 1)


def f2_mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t00 = f2_mul(a0, b0)
    t11 = f2_mul(a1, b1)
    t22 = f2_mul(a2, b2)
    c0 = f2_add(t00, f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(t22))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t11)
    return (c0, c1, c2)


def f6_mul_v(a):
    # (a0 + a1 v + a2 v^2) * v = xi a2 + a0 v + a1 v^2
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e: int):
    res = F12_ONE
    for bit in bin(e)[2:]:
        res = f12_sqr(res)
        if bit == "1":
            res = f12_mul(res, a)
    return res


def f12_from_fp(c: int):
    return (((c % P, 0), F2_ZERO, F2_ZERO), F6_ZERO)


def f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def f12_sub(a, b):
    return (f6_sub(a[0], b[0]), f6_sub(a[1], b[1]))


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


# w as an Fp12 element and the untwist constants: w^2 = v, w^6 = xi.
F12_W = (F6_ZERO, F6_ONE)


def untwist(Q):
    """E'(Fp2): y^2 = x^3 + 4 xi  ->  E(Fp12): y^2 = x^3 + 4,   (x, y) -> (x / w^2, y / w^3)."""
    x, y = Q
    w2 = f12_mul(F12_W, F12_W)
    w3 = f12_mul(w2, F12_W)
    xe = ((x, F2_ZERO, F2_ZERO), F6_ZERO)
    ye = ((y, F2_ZERO, F2_ZERO), F6_ZERO)
    return (f12_mul(xe, f12_inv(w2)), f12_mul(ye, f12_inv(w3)))


# ----------------------------------------------------------------------------------------------
# Curves.  Points are affine tuples; None is the point at infinity.
# ----------------------------------------------------------------------------------------------
G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)
B1 = 4
B2 = (4, 4)


def g1_on_curve(Pt) -> bool:
    if Pt is None:
        return True
    x, y = Pt
    return (y * y - x * x * x - B1) % P == 0


def g1_add(A, B):
    if A is None:
        return B
    if B is None:
        return A
    x1, y1 = A
    x2, y2 = B
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * inv(2 * y1) % P
    else:
        lam = (y2 - y1) * inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_neg(A):
    return None if A is None else (A[0], (-A[1]) % P)


def g1_mul(A, k: int):
    res = None
    for bit in bin(k)[2:] if k > 0 else "":
        res = g1_add(res, res)
        if bit == "1":
            res = g1_add(res, A)
    return res


def g2_on_curve(Pt) -> bool:
    if Pt is None:
        return True
    x, y = Pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_add(A, B):
    if A is None:
        return B
    if B is None:
        return A
    x1, y1 = A
    x2, y2 = B
    if x1 == x2:
        if f2_add(y1, y2) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def g2_neg(A):
    return None if A is None else (A[0], f2_neg(A[1]))


def g2_mul(A, k: int):
    res = None
    for bit in bin(k)[2:] if k > 0 else "":
        res = g2_add(res, res)
        if bit == "1":
            res = g2_add(res, A)
    return res


# ----------------------------------------------------------------------------------------------
# ZCash compressed serialization
# ----------------------------------------------------------------------------------------------
HALF_P = (P - 1) // 2


def g1_compress(Pt) -> bytes:
    if Pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = Pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if y > HALF_P:
        b[0] |= 0x20
    return bytes(b)


def g2_compress(Pt) -> bytes:
    if Pt is None:
        return bytes([0xC0]) + bytes(95)
    (x0, x1), (y0, y1) = Pt
    b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    b[0] |= 0x80
    big = (y1 > HALF_P) if y1 != 0 else (y0 > HALF_P)
    if big:
        b[0] |= 0x20
    return bytes(b)


def _flags(data: bytes):
    c = (data[0] >> 7) & 1
    i = (data[0] >> 6) & 1
    s = (data[0] >> 5) & 1
    return c, i, s


def g1_decompress(data: bytes, subgroup_check: bool = True):
    """Returns the point (None = infinity); raises BLSError on any invalid encoding."""
    if len(data) != 48:
        raise BLSError("bad length")
    c, i, s = _flags(data)
    if not c:
        raise BLSError("not compressed")
    body = bytearray(data)
    body[0] &= 0x1F
    if i:
        if s or any(body):
            raise BLSError("bad infinity encoding")
        return None
    x = int.from_bytes(body, "big")
    if x >= P:
        raise BLSError("non-canonical x")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise BLSError("not on curve")
    if (y > HALF_P) != bool(s):
        y = (-y) % P
    Pt = (x, y)
    if subgroup_check and g1_mul(Pt, R) is not None:
        raise BLSError("not in subgroup")
    return Pt


def g2_decompress(data: bytes, subgroup_check: bool = True):
    if len(data) != 96:
        raise BLSError("bad length")
    c, i, s = _flags(data)
    if not c:
        raise BLSError("not compressed")
    body = bytearray(data)
    body[0] &= 0x1F
    if i:
        if s or any(body):
            raise BLSError("bad infinity encoding")
        return None
    x1 = int.from_bytes(body[:48], "big")
    x0 = int.from_bytes(body[48:], "big")
    if x0 >= P or x1 >= P:
        raise BLSError("non-canonical x")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise BLSError("not on curve")
    big = (y[1] > HALF_P) if y[1] != 0 else (y[0] > HALF_P)
    if big != bool(s):
        y = f2_neg(y)
    Pt = (x, y)
    if subgroup_check and g2_mul(Pt, R) is not None:
        raise BLSError("not in subgroup")
    return Pt


# ----------------------------------------------------------------------------------------------
# RFC 9380 hash_to_curve for G2 (BLS12381G2_XMD:SHA-256_SSWU_RO_)
# ----------------------------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, s_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes):
    L = 64
    uniform = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(uniform[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


# E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def map_to_curve_sswu(u):
    """RFC 9380 section 6.6.2 (straight-line description, not the optimized one)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    tv1 = F2_ZERO if f2_is_zero(den) else f2_inv(den)
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x = x1
        y = f2_sqrt(gx1)
    else:
        x = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)
        y = f2_sqrt(gx2)
    assert y is not None
    if sgn0_fp2(u) != sgn0_fp2(y):
        y = f2_neg(y)
    return (x, y)


def _f2(c0: int, c1: int):
    return (c0 % P, c1 % P)


# RFC 9380 Appendix E.3 (3-isogeny E2' -> E2).  Self-checked in tests: the map lands on E2.
ISO3_XNUM = [
    _f2(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
        0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    _f2(0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    _f2(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
        0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    _f2(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO3_XDEN = [
    _f2(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    _f2(0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    _f2(1, 0),
]
ISO3_YNUM = [
    _f2(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
        0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    _f2(0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    _f2(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
        0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    _f2(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO3_YDEN = [
    _f2(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
        0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    _f2(0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    _f2(0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    _f2(1, 0),
]


def _poly_eval(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(Pt):
    if Pt is None:
        return None
    x, y = Pt
    xd = _poly_eval(ISO3_XDEN, x)
    yd = _poly_eval(ISO3_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xo = f2_mul(_poly_eval(ISO3_XNUM, x), f2_inv(xd))
    yo = f2_mul(y, f2_mul(_poly_eval(ISO3_YNUM, x), f2_inv(yd)))
    return (xo, yo)


def clear_cofactor_g2(Pt):
    return g2_mul(Pt, H_EFF_G2)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map_g2(map_to_curve_sswu(u0))
    q1 = iso_map_g2(map_to_curve_sswu(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ----------------------------------------------------------------------------------------------
# Pairing: affine Miller loop over generic Fp12, plain final exponentiation.
# ----------------------------------------------------------------------------------------------
FINAL_EXP = (P ** 12 - 1) // R


def _line(T, S, Pe):
    """Line through T and S (tangent when T == S), evaluated at Pe; all points in E(Fp12)."""
    (xt, yt), (xs, ys) = T, S
    xp, yp = Pe
    if T == S:
        num = f12_mul(f12_from_fp(3), f12_mul(xt, xt))
        den = f12_mul(f12_from_fp(2), yt)
    else:
        num = f12_sub(ys, yt)
        den = f12_sub(xs, xt)
    lam = f12_mul(num, f12_inv(den))
    return f12_sub(f12_sub(yp, yt), f12_mul(lam, f12_sub(xp, xt)))


def _e12_add(A, B):
    (x1, y1), (x2, y2) = A, B
    if A == B:
        lam = f12_mul(f12_mul(f12_from_fp(3), f12_mul(x1, x1)), f12_inv(f12_mul(f12_from_fp(2), y1)))
    else:
        lam = f12_mul(f12_sub(y2, y1), f12_inv(f12_sub(x2, x1)))
    x3 = f12_sub(f12_sub(f12_mul(lam, lam), x1), x2)
    y3 = f12_sub(f12_mul(lam, f12_sub(x1, x3)), y1)
    return (x3, y3)


def miller_loop(Pg1, Qg2):
    """f_{|x|,Q}(P), conjugated because x < 0 (vertical lines dropped: killed by the final exp)."""
    if Pg1 is None or Qg2 is None:
        return F12_ONE
    Qe = untwist(Qg2)
    Pe = (f12_from_fp(Pg1[0]), f12_from_fp(Pg1[1]))
    T = Qe
    f = F12_ONE
    for bit in bin(X_ABS)[3:]:
        f = f12_mul(f12_sqr(f), _line(T, T, Pe))
        T = _e12_add(T, T)
        if bit == "1":
            f = f12_mul(f, _line(T, Qe, Pe))
            T = _e12_add(T, Qe)
    return f12_conj(f)


def final_exponentiation(f):
    return f12_pow(f, FINAL_EXP)


def pairing(Pg1, Qg2):
    return final_exponentiation(miller_loop(Pg1, Qg2))


def pairing_product_is_one(pairs: Sequence[Tuple[object, object]]) -> bool:
    f = F12_ONE
    for Pg1, Qg2 in pairs:
        f = f12_mul(f, miller_loop(Pg1, Qg2))
    return final_exponentiation(f) == F12_ONE


# ----------------------------------------------------------------------------------------------
# Scalars (Fr) and the tbls.Implementation semantics (herumi.go)
# ----------------------------------------------------------------------------------------------
def sk_deserialize(sk: bytes) -> int:
    if len(sk) != 32:
        raise BLSError("bad secret length")
    v = int.from_bytes(sk, "big")
    if v >= R:
        raise BLSError("secret not in Fr")
    return v


def sk_serialize(v: int) -> bytes:
    return (v % R).to_bytes(32, "big")


def secret_to_public_key(sk: bytes) -> bytes:
    """herumi.go:67-80 (GetSafePublicKey rejects the zero secret)."""
    try:
        v = sk_deserialize(sk)
    except BLSError as e:
        raise BLSError("cannot unmarshal secret into Herumi secret key") from e
    if v == 0:
        raise BLSError("cannot obtain public key from secret")
    return g1_compress(g1_mul(G1_GEN, v))


def sign(sk: bytes, msg: bytes) -> bytes:
    """herumi.go:303-313: sigma = sk * H(msg)."""
    try:
        v = sk_deserialize(sk)
    except BLSError as e:
        raise BLSError("cannot unmarshal secret into Herumi secret key") from e
    return g2_compress(g2_mul(hash_to_g2(msg), v))


def _core_verify(pk_pt, msg: bytes, sig_pt) -> bool:
    if pk_pt is None:  # KeyValidate: identity public key rejected
        return False
    H = hash_to_g2(msg)
    return pairing_product_is_one([(pk_pt, H), (g1_neg(G1_GEN), sig_pt)])


def verify(pk: bytes, msg: bytes, sig: bytes) -> None:
    """herumi.go:285-301; raises BLSError with the reference's three error strings."""
    try:
        pk_pt = g1_decompress(pk)
    except BLSError as e:
        raise BLSError("cannot set compressed public key in Herumi format") from e
    try:
        sig_pt = g2_decompress(sig)
    except BLSError as e:
        raise BLSError("cannot unmarshal signature into Herumi signature") from e
    if not _core_verify(pk_pt, msg, sig_pt):
        raise BLSError("signature not verified")


def verify_status(pk: bytes, msg: bytes, sig: bytes) -> int:
    """0 ok, 1 bad public key encoding, 2 bad signature encoding, 3 not verified."""
    try:
        verify(pk, msg, sig)
        return 0
    except BLSError as e:
        s = str(e)
        if s.startswith("cannot set compressed public key"):
            return 1
        if s.startswith("cannot unmarshal signature"):
            return 2
        return 3


def lagrange_coeffs_at_zero(ids: Sequence[int]) -> List[int]:
    """lambda_i = prod_{j != i} x_j / (x_j - x_i)  mod r."""
    out = []
    for i, xi in enumerate(ids):
        num, den = 1, 1
        for j, xj in enumerate(ids):
            if j == i:
                continue
            num = num * xj % R
            den = den * (xj - xi) % R
        out.append(num * pow(den, -1, R) % R)
    return out


def threshold_aggregate(partials: Dict[int, bytes]) -> bytes:
    """herumi.go:244-283 (Sign.Recover at x = 0 with the share indices as ids)."""
    ids, pts = [], []
    for idx, sig in partials.items():
        try:
            pts.append(g2_decompress(sig))
        except BLSError as e:
            raise BLSError("cannot unmarshal signature into Herumi signature") from e
        ids.append(int(idx))
    if not ids or any(i % R == 0 for i in ids) or len(set(i % R for i in ids)) != len(ids):
        raise BLSError("cannot combine signatures")
    lam = lagrange_coeffs_at_zero(ids)
    acc = None
    for l, pt in zip(lam, pts):
        acc = g2_add(acc, g2_mul(pt, l))
    return g2_compress(acc)


def aggregate(sigs: Sequence[bytes]) -> bytes:
    """herumi.go:220-242: the only error path is deserialization; an empty list sums to infinity."""
    acc = None
    for s in sigs:
        try:
            acc = g2_add(acc, g2_decompress(s))
        except BLSError as e:
            raise BLSError("cannot unmarshal signature into Herumi signature") from e
    return g2_compress(acc)


def verify_aggregate(pks: Sequence[bytes], sig: bytes, msg: bytes) -> None:
    """herumi.go:315-339 (FastAggregateVerify)."""
    try:
        sig_pt = g2_decompress(sig)
    except BLSError as e:
        raise BLSError("cannot unmarshal signature into Herumi signature") from e
    pts = []
    for pk in pks:
        try:
            pts.append(g1_decompress(pk))
        except BLSError as e:
            raise BLSError("cannot set compressed public key in Herumi format") from e
    if not pts or any(p is None for p in pts):
        raise BLSError("signature verification failed")
    acc = None
    for p in pts:
        acc = g1_add(acc, p)
    if not _core_verify(acc, msg, sig_pt):
        raise BLSError("signature verification failed")


def threshold_split_poly(secret: int, poly_tail: Sequence[int], total: int) -> Dict[int, bytes]:
    """herumi.go:84-181: share_i = secret + sum_{j>=1} poly_j * i^j (mod r), i = 1..total."""
    poly = [secret] + list(poly_tail)
    out = {}
    for i in range(1, total + 1):
        acc = 0
        for c in reversed(poly):
            acc = (acc * i + c) % R
        out[i] = sk_serialize(acc)
    return out


def recover_secret(shares: Dict[int, bytes]) -> bytes:
    """herumi.go:183-218."""
    ids = [int(i) for i in shares]
    if not ids or any(i % R == 0 for i in ids) or len(set(ids)) != len(ids):
        raise BLSError("cannot recover full private key from partial keys")
    lam = lagrange_coeffs_at_zero(ids)
    acc = 0
    for l, (_, v) in zip(lam, shares.items()):
        acc = (acc + l * sk_deserialize(v)) % R
    return sk_serialize(acc)
