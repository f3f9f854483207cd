"""The gfx950 Montgomery product is hand-written asm (charon_amd/tools/gen_fp_asm.py), which the host
build never runs.  These CPU tests interpret the EMITTED instruction stream (the text inside
charon_amd/csrc/fp_asm_gfx950.h) lane-scalar and compare it with Python big-integer Montgomery
products, so a schedule change is checked here before it reaches a GPU.  The GPU parity tests then
cover it end to end through every curve and pairing result."""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "charon_amd", "tools"))
import gen_fp_asm as g  # noqa: E402

R_INV = pow(pow(2, 384, g.P), -1, g.P)


def _limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(12)]


def _val(limbs):
    return sum(v << (32 * i) for i, v in enumerate(limbs))


def _header_body():
    return _macro_body("BLS_FP_MUL_ASM_BODY")


def _cases(n, seed):
    rnd = random.Random(seed)
    edge = [0, 1, 2, g.P - 1, g.P - 2, (g.P - 1) // 2, (1 << 380), g.P - (1 << 32)]
    return edge + [rnd.randrange(g.P) for _ in range(n)]


def test_header_matches_generator():
    assert _header_body() == g.gen_mul(), "fp_asm_gfx950.h is stale: rerun charon_amd/tools/gen_fp_asm.py"


def test_product_schedule_is_montgomery():
    body = _header_body()
    cases = _cases(400, 7)
    rnd = random.Random(8)
    for a in cases:
        for b in (a, rnd.choice(cases)):
            got = _val(g.emulate(body, _limbs(a), _limbs(b)))
            assert got == a * b * R_INV % g.P, (hex(a), hex(b))


@pytest.mark.parametrize("chains,square", [(1, False), (2, False), (2, True)])
def test_radix29_experiment_is_montgomery(chains, square):
    """The measured-but-not-shipped radix-2^29 routine (R = 2^406, weakly reduced output, see the generator's
    docstring and profiles/r02_prod_probe.txt): scheduled stream == a*b/2^406 mod p, < 2p, for any 384-bit input."""
    body, _ = g.body_text(square=square, chains=chains, pool=("s[40:41]", "s[42:43]"))
    g.check(body, square=square, trials=120, seed=chains)


def _macro_body(name):
    text = open(os.path.join(ROOT, "charon_amd", "csrc", "fp_asm_gfx950.h")).read()
    block = text.split("#define %s \\" % name, 1)[1].split("\n\n", 1)[0]
    return [s.replace("\\n\\t", "") for s in re.findall(r'^\s+"([^"]*)"', block, re.M)]


@pytest.mark.parametrize("kind", ["add", "sub", "neg"])
def test_modular_add_sub_neg_blocks(kind):
    """The device fp_add / fp_sub / fp_neg asm blocks (field.h): emitted text == generator, and the interpreted
    stream equals (a +- b) mod p / -a mod p on canonical operands, edge values included."""
    name = {"add": "BLS_FP_ADD_ASM", "sub": "BLS_FP_SUB_ASM", "neg": "BLS_FP_NEG_ASM"}[kind]
    body = _macro_body(name)
    assert body == {"add": g.gen_add(), "sub": g.gen_sub(), "neg": g.gen_sub(neg=True)}[kind]
    cases = _cases(150, 21)
    rnd = random.Random(22)
    pl = _limbs(g.P)
    for a in cases:
        b = rnd.choice(cases)
        ins = {25 + i: v for i, v in enumerate(_limbs(a))}
        if kind == "neg":
            ins.update({37 + i: v for i, v in enumerate(pl)})
            want = (-a) % g.P
        else:
            ins.update({37 + i: v for i, v in enumerate(_limbs(b))})
            ins.update({49 + i: v for i, v in enumerate(pl)})
            want = (a + b) % g.P if kind == "add" else (a - b) % g.P
        got = _val(g.emulate_positional(body, list(range(12)), ins))
        assert got == want, (kind, hex(a), hex(b))


@pytest.mark.parametrize("kind", ["add_lazy", "sub_lazy"])
def test_lazy_add_sub_blocks(kind):
    """Unreduced product operands: a + b and a + (p - b), both in [0, 2p) for canonical a, b; and the product
    routine maps such operands (a*b < p*2^384) to the canonical Montgomery product."""
    name = {"add_lazy": "BLS_FP_ADD_LAZY_ASM", "sub_lazy": "BLS_FP_SUB_LAZY_ASM"}[kind]
    body = _macro_body(name)
    assert body == (g.gen_add_lazy() if kind == "add_lazy" else g.gen_sub_lazy())
    mul = _header_body()
    cases = _cases(120, 31)
    rnd = random.Random(32)
    pl = _limbs(g.P)
    for a in cases:
        b = rnd.choice(cases)
        if kind == "add_lazy":
            ins = {12 + i: v for i, v in enumerate(_limbs(a))}
            ins.update({24 + i: v for i, v in enumerate(_limbs(b))})
            want = a + b
        else:
            ins = {24 + i: v for i, v in enumerate(_limbs(a))}
            ins.update({36 + i: v for i, v in enumerate(_limbs(b))})
            ins.update({48 + i: v for i, v in enumerate(pl)})
            want = a + g.P - b
        got = _val(g.emulate_positional(body, list(range(12)), ins))
        assert got == want and got < 2 * g.P
        c = rnd.choice(cases)
        for x, y in ((got, got), (got, c), (c, got)):
            assert _val(g.emulate(mul, _limbs(x), _limbs(y))) == x * y * R_INV % g.P


def test_fp2_product_routine():
    """The device fp2_mul routine (BLS_FP2_MUL_ASM_BODY, gen_fp2_mul): emitted text == generator, and the interpreted
    stream gives c0 = (a0 b0 - a1 b1)/R, c1 = (a0 b1 + a1 b0)/R mod p, canonical, on canonical operands with edges
    (0, 1, p - 1: the final-subtraction boundaries), and on unreduced operands in [0, 2p) (lazy sums: p, 2p - 1);
    a0, a1, b0 come back unchanged (the C++ declares them input-only)."""
    body = _macro_body("BLS_FP2_MUL_ASM_BODY")
    assert body == g.gen_fp2_mul(), "fp_asm_gfx950.h is stale: rerun charon_amd/tools/gen_fp_asm.py"
    cases = _cases(60, 41) + [g.P, g.P + 1, 2 * g.P - 1, 2 * g.P - 2, g.P + (1 << 300)]
    rnd = random.Random(42)
    for t in range(300):
        a0, a1, b0, b1 = (rnd.choice(cases) for _ in range(4))
        regs = {}
        for base, x in ((g.FP2_A0, a0), (g.FP2_A1, a1), (g.FP2_B0, b0), (g.FP2_B1, b1)):
            regs.update({base + j: v for j, v in enumerate(_limbs(x))})
        g.emulate(body, None, None, regs)
        c0 = _val([regs[g.FP2_C0 + j] for j in range(12)])
        c1 = _val([regs[g.FP2_C1 + j] for j in range(12)])
        assert c0 == (a0 * b0 - a1 * b1) * R_INV % g.P, (t, hex(a0), hex(a1), hex(b0), hex(b1))
        assert c1 == (a0 * b1 + a1 * b0) * R_INV % g.P, (t, hex(a0), hex(a1), hex(b0), hex(b1))
        for base, x in ((g.FP2_A0, a0), (g.FP2_A1, a1), (g.FP2_B0, b0)):
            assert _val([regs[base + j] for j in range(12)]) == x


def test_fp2_square_routine():
    """The device fp2_sqr routine (BLS_FP2_SQR_ASM_BODY, gen_fp2_sqr): c0 = (a0^2 - a1^2)/R, c1 = 2 a0 a1/R mod p,
    canonical, on canonical operands with edges."""
    body = _macro_body("BLS_FP2_SQR_ASM_BODY")
    assert body == g.gen_fp2_sqr(), "fp_asm_gfx950.h is stale: rerun charon_amd/tools/gen_fp_asm.py"
    cases = _cases(60, 51)
    rnd = random.Random(52)
    for t in range(300):
        a0, a1 = rnd.choice(cases), rnd.choice(cases)
        regs = {g.FP2S_A0 + j: v for j, v in enumerate(_limbs(a0))}
        regs.update({g.FP2S_A1 + j: v for j, v in enumerate(_limbs(a1))})
        g.emulate(body, None, None, regs)
        c0 = _val([regs[g.FP2S_C0 + j] for j in range(12)])
        c1 = _val([regs[g.FP2S_C1 + j] for j in range(12)])
        assert c0 == (a0 * a0 - a1 * a1) * R_INV % g.P, (t, hex(a0), hex(a1))
        assert c1 == 2 * a0 * a1 * R_INV % g.P, (t, hex(a0), hex(a1))


@pytest.mark.parametrize("half", [0, 1])
def test_fp2_product_half_routine(half):
    """The split-Fp2 build's product half (BLS_FP2_MUL_HALF_ASM_BODY, gen_fp2_mul_half): with the lane mask in v76
    (0 or ~0) the interpreted stream gives c0 = (a0 b0 - a1 b1)/R or c1 = (a0 b1 + a1 b0)/R mod p, canonical, on
    canonical and unreduced operands in [0, 2p); a0, a1 come back unchanged."""
    body = _macro_body("BLS_FP2_MUL_HALF_ASM_BODY")
    assert body == g.gen_fp2_mul_half(), "fp_asm_gfx950.h is stale: rerun charon_amd/tools/gen_fp_asm.py"
    cases = _cases(60, 61) + [g.P, g.P + 1, 2 * g.P - 1, 2 * g.P - 2, g.P + (1 << 300)]
    rnd = random.Random(62 + half)
    for t in range(250):
        a0, a1, b0, b1 = (rnd.choice(cases) for _ in range(4))
        regs = {g.FP2H_MASK: 0xFFFFFFFF if half else 0}
        for base, x in ((0, a0), (12, a1), (24, b0), (36, b1)):
            regs.update({base + j: v for j, v in enumerate(_limbs(x))})
        g.emulate(body, None, None, regs)
        c = _val([regs[g.FP2H_OUT + j] for j in range(12)])
        want = (a0 * b1 + a1 * b0) if half else (a0 * b0 - a1 * b1)
        assert c == want * R_INV % g.P, (t, hex(a0), hex(a1), hex(b0), hex(b1))
        for base, x in ((0, a0), (12, a1)):
            assert _val([regs[base + j] for j in range(12)]) == x


@pytest.mark.parametrize("half", [0, 1])
def test_fp2_square_half_routine(half):
    """The split-Fp2 build's square half (BLS_FP2_SQR_HALF_ASM_BODY): c0 = (a0^2 - a1^2)/R or c1 = 2 a0 a1/R mod p,
    canonical, on canonical operands with edges; a0, a1 come back unchanged."""
    body = _macro_body("BLS_FP2_SQR_HALF_ASM_BODY")
    assert body == g.gen_fp2_sqr_half(), "fp_asm_gfx950.h is stale: rerun charon_amd/tools/gen_fp_asm.py"
    cases = _cases(60, 71)
    rnd = random.Random(72 + half)
    for t in range(250):
        a0, a1 = rnd.choice(cases), rnd.choice(cases)
        regs = {g.FP2H_MASK: 0xFFFFFFFF if half else 0}
        regs.update({j: v for j, v in enumerate(_limbs(a0))})
        regs.update({12 + j: v for j, v in enumerate(_limbs(a1))})
        g.emulate(body, None, None, regs)
        c = _val([regs[g.FP2HS_OUT + j] for j in range(12)])
        want = 2 * a0 * a1 if half else a0 * a0 - a1 * a1
        assert c == want * R_INV % g.P, (t, hex(a0), hex(a1))
        for base, x in ((0, a0), (12, a1)):
            assert _val([regs[base + j] for j in range(12)]) == x


def test_fp2_sum_of_products_routine():
    """The lazy-reduction experiment's routine (BLS_FP2_MUL2_ASM_BODY, gen_fp2_mul2): c = x y + z w
    with one Montgomery reduction per coefficient over four products, canonical on canonical operands (edges at the
    final subtraction's boundary included); x0, x1, y0, z0, z1, w0 come back unchanged."""
    body = g.gen_fp2_mul2()  # generated on demand (gen_fp_asm.py --lazy), not shipped in fp_asm_gfx950.h
    cases = _cases(60, 51)
    rnd = random.Random(52)
    for t in range(300):
        x0, x1, y0, y1, z0, z1, w0, w1 = (rnd.choice(cases) for _ in range(8))
        if t < 4:  # the largest sums the bound allows: every operand p - 1
            x0 = x1 = y0 = z0 = z1 = w0 = g.P - 1
            y1 = w1 = 0 if t & 1 else g.P - 1
        regs = {}
        for base, v in ((0, x0), (12, x1), (24, y0), (36, y1), (g.FP2M2_Z0, z0), (g.FP2M2_Z1, z1),
                        (g.FP2M2_W0, w0), (g.FP2M2_W1, w1)):
            regs.update({base + j: u for j, u in enumerate(_limbs(v))})
        g.emulate(body, None, None, regs)
        c0 = _val([regs[g.FP2_C0 + j] for j in range(12)])
        c1 = _val([regs[g.FP2_C1 + j] for j in range(12)])
        assert c0 == (x0 * y0 - x1 * y1 + z0 * w0 - z1 * w1) * R_INV % g.P, t
        assert c1 == (x0 * y1 + x1 * y0 + z0 * w1 + z1 * w0) * R_INV % g.P, t
        for base, v in ((0, x0), (12, x1), (24, y0), (g.FP2M2_Z0, z0), (g.FP2M2_Z1, z1), (g.FP2M2_W0, w0)):
            assert _val([regs[base + j] for j in range(12)]) == v


def test_fp2_sum_of_three_products_routine():
    """BLS_FP2_MUL3_ASM_BODY (gen_fp2_mul3): c = x y + z w + u t, one reduction per coefficient over six products,
    canonical on canonical operands, including all operands p - 1 (the largest sums)."""
    body = g.gen_fp2_mul3()
    cases = _cases(60, 61)
    rnd = random.Random(62)
    for t in range(200):
        v = [rnd.choice(cases) for _ in range(12)]
        if t < 4:
            v = [g.P - 1] * 12
            if t & 1:
                v[3] = v[7] = v[11] = 0
        x0, x1, y0, y1, z0, z1, w0, w1, u0, u1, t0, t1 = v
        regs = {}
        for base, val in ((0, x0), (12, x1), (24, y0), (36, y1), (g.FP2M2_Z0, z0), (g.FP2M2_Z1, z1),
                          (g.FP2M2_W0, w0), (g.FP2M2_W1, w1), (g.FP2M3_U0, u0), (g.FP2M3_U1, u1),
                          (g.FP2M3_T0, t0), (g.FP2M3_T1, t1)):
            regs.update({base + j: u for j, u in enumerate(_limbs(val))})
        g.emulate(body, None, None, regs)
        c0 = _val([regs[g.FP2_C0 + j] for j in range(12)])
        c1 = _val([regs[g.FP2_C1 + j] for j in range(12)])
        assert c0 == (x0 * y0 - x1 * y1 + z0 * w0 - z1 * w1 + u0 * t0 - u1 * t1) * R_INV % g.P, t
        assert c1 == (x0 * y1 + x1 * y0 + z0 * w1 + z1 * w0 + u0 * t1 + u1 * t0) * R_INV % g.P, t
