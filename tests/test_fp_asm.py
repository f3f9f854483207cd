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


# ---------------------------------------------------------------- carry elision (round 6)
def _symbolic_max(body, bound, carried="v[38:39]"):
    """Walks a product stream with every operand at its largest value: a mad that no v_addc follows must leave the
    64-bit accumulator <= 2^64 - 1 (the column's carried value counts as (carries + 1) 2^32).  Independent of the
    generator's own bookkeeping (_comba); returns the number of carry-free mads."""
    free, acc, n_cur, n_prev = 0, 0, 0, 0
    for k, ins in enumerate(body):
        op, rest = ins.split(" ", 1)
        o = [t.strip() for t in rest.split(",")]
        if op != "v_mad_u64_u32":
            continue
        if o[4] == "0":
            base = 0
        elif o[4] == carried:
            n_prev, n_cur = n_cur, 0
            base = (n_prev + 1) << 32
        else:
            base = acc
        val = base + bound(o[2]) * bound(o[3])
        if body[k + 1].startswith("v_addc_co_u32") if k + 1 < len(body) else False:
            n_cur += 1
            acc = (1 << 64) - 1  # caught: only the accumulator's width is known from here on
        else:
            assert val <= (1 << 64) - 1, (k, ins, hex(val))
            free += 1
            acc = val
    return free


def test_product_carry_elision_is_sound():
    """gen_mul's carry-free mads: with operands < 2^382 (top limb < 2^30), q digits < 2^32 and p's limbs exact, no
    carry-free mad can overflow its accumulator; and the same for a two-product column schedule (the Fp2 routines)."""
    pl = {"s%d" % (16 + j): (g.P >> (32 * j)) & 0xFFFFFFFF for j in range(12)}

    def bound_for(tops):
        return lambda r: pl[r] if r in pl else (g.TOP_BOUND if r in tops else 0xFFFFFFFF)

    body = g.gen_mul()
    free = _symbolic_max(body, bound_for({"v11", "v23"}))
    assert free >= 70 and sum(x.startswith("v_addc") for x in body) == 288 - free + 0
    w = []
    V = lambda base: (lambda j: "v%d" % (base + j))
    g._comba(w.append, [(V(100), V(112)), (V(124), V(136))], V(148), V(148), 48)
    assert _symbolic_max(w, bound_for({"v111", "v123", "v135", "v147"}), carried="v[50:51]") >= 70


def test_product_extreme_operands_keep_every_carry():
    """Operands at the elision's limits (2^382 - 1, every lower limb all ones, the top limb at 2^30 - 1 or at 2p's) in
    the strict interpreter: no mad drops a carry, and the products stay Montgomery products (canonical for the Fp
    product, whose operands may be anything < 2^382)."""
    top = (1 << 382) - 1
    ext = [top, top - 1, (0x3FFFFFFF << 352), (1 << 352) - 1, 2 * g.P - 1, 2 * g.P, g.P - 1, 0, 1,
           (0x340223D4 << 352) | ((1 << 352) - 1)]
    rnd = random.Random(606)
    mul = g.gen_mul()
    for a in ext:
        for b in ext + [rnd.randrange(1 << 382) for _ in range(4)]:
            got = _val(g.emulate(mul, _limbs(a), _limbs(b)))
            assert got == a * b * R_INV % g.P, (hex(a), hex(b))
    f2m, ok = g.gen_fp2_mul(), [x for x in ext if x <= 2 * g.P]
    for t in range(200):
        a0, a1, b0 = (rnd.choice(ext) for _ in range(3))
        b1 = rnd.choice(ok)  # the routine forms 2p - b1
        regs = {}
        for base, x in ((g.FP2_A0, a0), (g.FP2_A1, a1), (g.FP2_B0, b0), (g.FP2_B1, b1)):
            regs.update({base + j: v for j, v in enumerate(_limbs(x))})
        g.emulate(f2m, None, None, regs)
        c0 = _val([regs[g.FP2_C0 + j] for j in range(12)])
        c1 = _val([regs[g.FP2_C1 + j] for j in range(12)])
        assert c0 % g.P == (a0 * b0 - a1 * b1) * R_INV % g.P and c1 % g.P == (a0 * b1 + a1 * b0) * R_INV % g.P


def test_strict_interpreter_catches_a_dropped_carry():
    """The checker is live: removing a carry-catching v_addc from gen_mul makes the interpreter raise on all-ones
    operands."""
    body = g.gen_mul()
    ks = [i for i, x in enumerate(body) if x.startswith("v_addc_co_u32_e32")]
    k = ks[len(ks) // 2]  # a mid-product column: all-ones operands set its carries
    broken = body[:k] + body[k + 1:]
    a = (1 << 382) - 1
    with pytest.raises(g.DroppedCarry):
        g.emulate(broken, _limbs(a), _limbs(a))
