"""Generate charon_amd/csrc/fp_asm_gfx950.h: the gfx950 Montgomery product as one asm routine.

SHIPPED (gen_mul): radix 2^32, 12 limbs, product scanning (Comba) with the Montgomery reduction
interleaved per column.  Every limb product is one v_mad_u64_u32 into a 64-bit column accumulator,
plus one v_addc_co_u32 catching the carry into a third word unless the column's bound proves the
accumulator cannot overflow there (carry elision, _comba: 74 of the 288 carries), + 12 v_mul_lo_u32,
canonical output (final conditional subtraction of p); 598 instructions (672 with every carry caught).  Registers are pinned (a = v[0:11] in/out, b = v[12:23])
and only v24-v39, s16-s28 and vcc are clobbered, so values live across a product stay in registers.
The final select uses v_cndmask_b32_e64 with an explicit VCC operand: on gfx950 the VOP2 (e32) form that
reads VCC implicitly issues at ~19 cycles per instruction against ~4.4 for the e64 form and for v_bfi_b32
(profiles/r02_prod_probe.txt, tools/sel_probe.hip).

EXPERIMENT (gen_mul29, not emitted): radix 2^29, 14 limbs, R = 2^406, no carry capture (a column of
<= 28 terms < 2^58 fits the 64-bit accumulator), two accumulator chains, lazy [0, 2p) output, list
scheduled.  Measured on MI355X (tools/prod_probe.hip): at one wave per SIMD -- the C2 regime -- it is no
faster (2,802-2,946 vs 2,754 cycles per product: v_mad_u64_u32 issues at 5 cycles for one wave, so 392
mads cost what 288 mads + 288 addc cost); at 2 and 4 waves per SIMD it is 10-14 % faster.  Adopting it
also needs R = 2^406 constants and a weakly reduced value domain everywhere, so it stays an experiment.

Correctness: `emulate()` interprets an emitted stream on the CPU; tests/test_fp_asm.py checks the shipped
routine (and the experiment) against big-integer Montgomery products before any GPU run.

Run:  python3 charon_amd/tools/gen_fp_asm.py
"""
import os
import random

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
N32 = 12
W = 29
N = 14
MASK = (1 << W) - 1
R_MONT = 1 << (W * N)  # 2^406
PINV29 = (-pow(P, -1, 1 << W)) % (1 << W)
P29 = [(P >> (W * i)) & MASK for i in range(N)]
assert P29[13] == 13 and 4 * P < R_MONT

# ---------------------------------------------------------------- register map
A = lambda k: "v%d" % k if k < 12 else "v%d" % (24 + k - 12)
B = lambda k: "v%d" % (12 + k) if k < 12 else "v%d" % (26 + k - 12)
M = lambda k: "v%d" % (28 + k)
C0 = (42, 43)
CB = [(44, 45), (46, 47)]
VPINV = "v48"
SP = lambda k: "s%d" % (16 + k) if k < 13 else "13"
CLOBBER_V = list(range(12, 49))
CLOBBER_S = list(range(16, 29))


def pair(r):
    return "v[%d:%d]" % r


class Ins:
    __slots__ = ("text", "defs", "uses", "lat", "salu")

    def __init__(self, text, defs, uses, lat=8, salu=False):
        self.text, self.defs, self.uses, self.lat, self.salu = text, set(defs), set(uses), lat, salu


def regs_of(op):
    """Register names an operand string touches (v/s, pairs expanded)."""
    op = op.strip()
    if op.startswith("v["):
        lo, hi = op[2:-1].split(":")
        return ["v%d" % i for i in range(int(lo), int(hi) + 1)]
    if op.startswith("s[") :
        lo, hi = op[2:-1].split(":")
        return ["s%d" % i for i in range(int(lo), int(hi) + 1)]
    if (op.startswith("v") or op.startswith("s")) and op[1:].isdigit():
        return [op]
    return []


def I(text, dst, srcs, lat=8):
    defs = regs_of(dst)
    uses = [r for s in srcs for r in regs_of(s)]
    return Ins(text, defs, uses, lat)


SDST_POOL = ["vcc"]  # carry-out destinations of the mads (never read); rotated
_sdst_next = [0]


def mad(acc, x, y, src2=None):
    s2 = pair(acc) if src2 is None else src2
    srcs = [x, y] + ([s2] if src2 is None else [])
    sd = SDST_POOL[_sdst_next[0] % len(SDST_POOL)]
    _sdst_next[0] += 1
    # the carry-out is never read: not tracked as a dependency
    return I("v_mad_u64_u32 %s, %s, %s, %s, %s" % (pair(acc), sd, x, y, s2), pair(acc), srcs, lat=8)


def gen_mul29(square=False, chains=2):
    """Returns the list of Ins (unscheduled, in a valid program order)."""
    out = []
    for k in range(13):
        out.append(Ins("s_mov_b32 %s, 0x%08x" % (SP(k), P29[k]), [SP(k)], [], lat=1))
    out.append(I("v_mov_b32 %s, 0x%08x" % (VPINV, PINV29), VPINV, [], lat=4))

    def convert(R, base):
        # 12x32 (registers base..base+11) -> 14x29 in R(k), high limb first (in place)
        for k in range(N - 1, -1, -1):
            o = W * k
            w, s = o // 32, o % 32
            src = lambda j: "v%d" % (base + j)
            if w + 1 >= N32:  # top limb: the remaining bits of word 11
                out.append(I("v_lshrrev_b32 %s, %d, %s" % (R(k), s, src(w)), R(k), [src(w)], lat=4))
            elif s + W <= 32:
                out.append(I("v_bfe_u32 %s, %s, %d, %d" % (R(k), src(w), s, W), R(k), [src(w)], lat=4))
            else:
                out.append(I("v_alignbit_b32 %s, %s, %s, %d" % (R(k), src(w + 1), src(w), s), R(k),
                             [src(w + 1), src(w)], lat=4))
                out.append(I("v_and_b32_e32 %s, 0x%08x, %s" % (R(k), MASK, R(k)), R(k), [R(k)], lat=4))

    Bk = A if square else B
    if not square:
        convert(B, 12)
    convert(A, 0)

    started = {C0: False}

    def add_term(acc, x, y):
        if not started.get(acc, False):
            out.append(mad(acc, x, y, src2="0"))
            started[acc] = True
        else:
            out.append(mad(acc, x, y))

    for i in range(2 * N - 1):
        terms = []
        for j in range(max(0, i - N + 1), min(i, N - 1) + 1):
            terms.append((A(j), Bk(i - j)))
        for j in range(max(0, i - N + 1), min(i - 1, N - 1) + 1):
            terms.append((M(j), SP(i - j)))
        if i < N:
            # the quotient term m_i * p_0 comes last; keep a * b_0 in the list
            pass
        cb = CB[i % 2]
        started[cb] = False
        accs = [C0, cb] if chains >= 2 else [C0]
        for t, (x, y) in enumerate(terms):
            add_term(accs[t % len(accs)], x, y)
        if chains >= 2 and started[cb]:
            out.append(I("v_lshl_add_u64 %s, %s, 0, %s" % (pair(C0), pair(cb), pair(C0)), pair(C0),
                         [pair(cb), pair(C0)], lat=8))
        lo = "v%d" % C0[0]
        if i < N:
            out.append(I("v_mul_lo_u32 %s, %s, %s" % (M(i), lo, VPINV), M(i), [lo, VPINV], lat=8))
            out.append(I("v_and_b32_e32 %s, 0x%08x, %s" % (M(i), MASK, M(i)), M(i), [M(i)], lat=4))
            out.append(mad(C0, M(i), SP(0)))
        else:
            out.append(I("v_and_b32_e32 %s, 0x%08x, %s" % (M(i - N), MASK, lo), M(i - N), [lo], lat=4))
        out.append(I("v_lshrrev_b64 %s, %d, %s" % (pair(C0), W, pair(C0)), pair(C0), [pair(C0)], lat=8))
    out.append(I("v_mov_b32 %s, v%d" % (M(N - 1), C0[0]), M(N - 1), ["v%d" % C0[0]], lat=4))
    # repack r (14 x 29 in M(0..13)) into 12 x 32 words in v0..v11
    for wd in range(N32):
        o = 32 * wd
        k, s = o // W, o % W
        dst = "v%d" % wd
        if s == 0:
            out.append(I("v_lshl_or_b32 %s, %s, %d, %s" % (dst, M(k + 1), W, M(k)), dst, [M(k + 1), M(k)], lat=4))
        else:
            out.append(I("v_lshrrev_b32 %s, %d, %s" % (dst, s, M(k)), dst, [M(k)], lat=4))
            out.append(I("v_lshl_or_b32 %s, %s, %d, %s" % (dst, M(k + 1), W - s, dst), dst, [M(k + 1), dst], lat=4))
            if W - s + W < 32:
                out.append(I("v_lshl_or_b32 %s, %s, %d, %s" % (dst, M(k + 2), 2 * W - s, dst), dst,
                             [M(k + 2), dst], lat=4))
    return out


def schedule(ins, issue=4):
    """Greedy list scheduler over true/anti/output register dependencies.  Priority = longest
    latency-weighted path to the end (critical path first).  Returns (ordered ins, modeled cycles)."""
    n = len(ins)
    succ = [[] for _ in range(n)]
    npred = [0] * n
    last_def, last_uses = {}, {}
    edges = set()

    def edge(a, b, lat):
        if (a, b) in edges:
            return
        edges.add((a, b))
        succ[a].append((b, lat))
        npred[b] += 1

    for i, x in enumerate(ins):
        for r in x.uses:                   # RAW
            if r in last_def:
                edge(last_def[r], i, ins[last_def[r]].lat)
        for r in x.defs:
            if r in last_def:              # WAW
                edge(last_def[r], i, 1)
            for u in last_uses.get(r, ()):  # WAR
                if u != i:
                    edge(u, i, 1)
        for r in x.uses:
            last_uses.setdefault(r, []).append(i)
        for r in x.defs:
            last_def[r] = i
            last_uses[r] = []
    prio = [0] * n
    for i in range(n - 1, -1, -1):
        prio[i] = max([l + prio[j] for j, l in succ[i]] + [ins[i].lat])
    ready_at = [0] * n
    avail = [i for i in range(n) if npred[i] == 0]
    order, t = [], 0
    while avail:
        # among instructions whose operands are ready at t, the highest priority; else the earliest
        cands = [i for i in avail if ready_at[i] <= t]
        if not cands:
            t = min(ready_at[i] for i in avail)
            continue
        i = max(cands, key=lambda j: (prio[j], -j))
        avail.remove(i)
        order.append(ins[i])
        t += 1 if ins[i].salu else issue
        for j, l in succ[i]:
            ready_at[j] = max(ready_at[j], t - issue + l if not ins[i].salu else t + l)
            npred[j] -= 1
            if npred[j] == 0:
                avail.append(j)
    assert len(order) == n
    return order, t


# ---------------------------------------------------------------- carry elision (round 6)
# A v_mad_u64_u32 needs its carry-out caught only when the 64-bit column accumulator can overflow.  Every product
# operand is < 2^382 (canonical values and the lazy sums in [0, 2p) of field.h), so a product with an operand's top
# limb is < 2^62, and p's limbs 3, 5 and 7-11 are well below 2^32.  Such terms go first in their column, right after
# the carried-in value (< (carries + 1) 2^32), and skip the v_addc while the sum of their bounds stays below 2^64.
# emulate(strict=True) raises when a mad drops a carry.
OPERAND_BITS = 382
ELIDE = True  # False: the round-5 streams (every carry caught)
P_MOV64 = True  # False: p staged with twelve v_mov_b32
P_SGPR = True  # False: every routine loads p and -p^-1 into s16-s28 itself (thirteen s_mov_b32)
ACC_IN_PLACE = True  # False: every result column's low word is moved out of v[acc:acc+1]
TOP_BOUND = (1 << (OPERAND_BITS - 352)) - 1  # an operand's top limb
LIMB_MAX = 0xFFFFFFFF
M64 = (1 << 64) - 1
PL32 = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]


def _comba(w, pairs, M, out, acc, elide=True):
    """Product scanning with the Montgomery reduction interleaved per column (radix 2^32, R = 2^384): appends
    r = (sum of X*Y over pairs)/R, raw, to the stream w.  pairs = [(X, Y)] (limb index -> register); M(i) holds the
    quotient digits; out(j) receives result limb j (from column j + 12; out(j) may alias a register dead by then).
    Accumulator v[acc:acc+1], the carried value (hi, carries) in v[acc+2:acc+3]; p in s16-s27, -p^-1 mod 2^32 in s28.
    elide=False: every mad catches its carry (the round-5 streams, term for term)."""
    lo, hi, mv, cw = ("v%d" % (acc + k) for k in range(4))
    accp, srcp = "v[%d:%d]" % (acc, acc + 1), "v[%d:%d]" % (acc + 2, acc + 3)
    Sp = lambda j: "s%d" % (16 + j)
    n_prev = 0
    for i in range(2 * N32 - 1):
        body = []
        for j in range(max(0, i - N32 + 1), min(i, N32 - 1) + 1):
            for X, Y in pairs:
                bx = TOP_BOUND if j == N32 - 1 else LIMB_MAX
                by = TOP_BOUND if i - j == N32 - 1 else LIMB_MAX
                body.append((X(j), Y(i - j), bx * by))
            if j < i:
                body.append((M(j), Sp(i - j), LIMB_MAX * PL32[i - j]))
        start = 0 if i == 0 else (n_prev + 1) << 32
        # Even result columns accumulate in place: the pair (out(i - 12), out(i - 11)) is the accumulator, so the
        # column's low word is already result limb i - 12 (no move).  out(i - 11) is read by exactly one term of the
        # column (its last use) -- that term goes first, before the first mad overwrites the register.
        cacc = accp
        alias = None
        if elide and ACC_IN_PLACE and i >= N32 and i % 2 == 0:
            lo_n, hi_n = int(out(i - N32)[1:]), int(out(i - N32 + 1)[1:])
            if lo_n % 2 == 0 and hi_n == lo_n + 1:
                ka = [k for k, t in enumerate(body) if out(i - N32 + 1) in (t[0], t[1])]
                assert len(ka) == 1, (i, ka)
                alias = ka[0]
                cacc = "v[%d:%d]" % (lo_n, hi_n)
        if elide:
            free, s = [], start
            order = sorted(range(len(body)), key=lambda k: body[k][2])
            if alias is not None:
                order = [alias] + [k for k in order if k != alias]
            for k in order:
                if s + body[k][2] > M64:
                    break
                free.append(k)
                s += body[k][2]
            assert alias is None or free[:1] == [alias], (i, "the in-place column's first term must be carry-free")
            seq = [(body[k], False) for k in free] + [(body[k], True) for k in range(len(body)) if k not in free]
        else:
            seq = [(t, not (i == 0 and k == 0)) for k, t in enumerate(body)]
            s = None
        st = {"src": "0" if i == 0 else srcp, "init": False, "n": 0}

        def mac(x, y, need):
            w("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (cacc, x, y, st["src"]))
            st["src"] = cacc
            if not need:
                return
            if st["init"]:
                w("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (cw, cw))
            else:
                w("v_addc_co_u32_e64 %s, vcc, 0, 0, vcc" % cw)
                st["init"] = True
            st["n"] += 1

        for k, ((x, y, _), need) in enumerate(seq):
            mac(x, y, need)
            if not elide and i == 0 and k == 0:
                w("v_mov_b32 %s, 0" % cw)
                st["init"] = True
        if i < N32:
            w("v_mul_lo_u32 %s, %s, s28" % (M(i), lo))
            b = LIMB_MAX * PL32[0]
            need = not elide or any(nd for _, nd in seq) or s + b > M64
            mac(M(i), Sp(0), need)
        if i == 2 * N32 - 2:
            if alias is not None:
                pass  # limbs 10 and 11 are the accumulator
            elif elide:
                w("v_mov_b32 %s, %s" % (out(i - N32), lo))
                w("v_mov_b32 %s, %s" % (out(N32 - 1), hi))
            else:
                w("v_mov_b32 %s, %s" % (out(i - N32), lo))
                w("v_mov_b32 %s, %s" % (mv, hi))
                w("v_mov_b32 %s, %s" % (out(N32 - 1), mv))
            break
        if not st["init"]:
            w("v_mov_b32 %s, 0" % cw)  # no carry caught in this column: the carried value's high word is 0
        if alias is not None:
            w("v_mov_b32 %s, %s" % (mv, out(i - N32 + 1)))
        else:
            if i >= N32:
                w("v_mov_b32 %s, %s" % (out(i - N32), lo))
            w("v_mov_b32 %s, %s" % (mv, hi))
        n_prev = st["n"]


def _p_sgprs(w):
    """p into s16-s27 and -p^-1 mod 2^32 into s28, or nothing with P_SGPR: the callers then hold them there (field.h
    BLS_P_SGPR_IN: loaded once from constant memory, inputs of every routine call, never clobbered), and the thirteen
    scalar moves -- a full issue slot each at one wave per SIMD (tools/isa_probe.hip) -- leave every call."""
    if P_SGPR:
        return
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    for j in range(N32):
        w("s_mov_b32 s%d, 0x%08x" % (16 + j, PL32[j]))
    w("s_mov_b32 s28, 0x%08x" % PINV32)


def _load_p(w, R):
    """p (s16-s27) into the VGPRs R(0..11): six v_mov_b64 from SGPR pairs (one issue slot per two limbs; every
    instruction of a one-wave-per-SIMD stream costs the same slot, tools/isa_probe.hip), or twelve v_mov_b32 with
    P_MOV64 = False."""
    if not P_MOV64:
        for j in range(N32):
            w("v_mov_b32 %s, s%d" % (R(j), 16 + j))
        return
    for j in range(0, N32, 2):
        lo = int(R(j)[1:])
        assert lo % 2 == 0 and R(j + 1) == "v%d" % (lo + 1)
        w("v_mov_b64 v[%d:%d], s[%d:%d]" % (lo, lo + 1, 16 + j, 17 + j))


# ---------------------------------------------------------------- old radix-2^32 routine (probe)
def gen_mul(e64_select=True, elide=None):
    """The shipped routine (Comba, radix 2^32, R = 2^384, canonical output for operands < 2^382): mad + addc carry
    capture except where the column bound makes the carry impossible (_comba).  e64_select=False, elide=False
    reproduce the round-1 stream (VOP2 v_cndmask_b32_e32, every carry caught) for the microbenchmark."""
    elide = ELIDE if elide is None else elide
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    Aa = lambda j: "v%d" % j
    Bb = lambda j: "v%d" % (12 + j)
    Mm = lambda j: "v%d" % (24 + j)
    Sp = lambda j: "s%d" % (16 + j)
    out = []
    w = out.append
    _p_sgprs(w)
    _comba(w, [(Aa, Bb)], Mm, Aa, 36, elide)
    _load_p(w, Mm)
    w("v_sub_co_u32_e32 v12, vcc, v0, v24")
    for j in range(1, N32):
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (Bb(j), Aa(j), Mm(j)))
    for j in range(N32):
        if e64_select:
            w("v_cndmask_b32_e64 %s, %s, %s, vcc" % (Aa(j), Bb(j), Aa(j)))
        else:
            w("v_cndmask_b32_e32 %s, %s, %s, vcc" % (Aa(j), Bb(j), Aa(j)))
    return out


gen_mul32 = gen_mul  # name used by tools/gen_probe_bodies.py


# ---------------------------------------------------------------- Fp2 product as two sums of products
# (a0 + a1 u)(b0 + b1 u) = (a0 b0 - a1 b1) + (a0 b1 + a1 b0) u.  Each coefficient is ONE Montgomery reduction
# of a sum of two 768-bit products (product scanning, reduction interleaved per column, as gen_mul):
#   c1 = (a0 b1 + a1 b0) / R,   c0 = (a0 b0 + a1 (2p - b1)) / R   (mod p)
# 2 x 432 mads instead of the 3 x 288 of Karatsuba with three reduced products, and no Fp additions: the
# Karatsuba sums, the three subtractions and one of the three final subtractions disappear.  Operands may be
# unreduced sums in [0, 2p): each sum of products is then < 8p^2 and (T + mp)/R < 8p^2/R + p < 1.82p, so one
# conditional subtraction still makes each output canonical.
# Registers: a0 = v[0:11], a1 = v[12:23], b0 = v[24:35] (preserved), b1 = v[36:47] (clobbered); c1 -> v[52:63],
# c0 -> v[64:75]; v48-v51, v76-v87, s16-s28 and vcc clobbered.
FP2_A0, FP2_A1, FP2_B0, FP2_B1, FP2_C1, FP2_C0, FP2_T = 0, 12, 24, 36, 52, 64, 76


def _gen_sop(w, X, Y, Z, Wd, M):
    """Appends r = (X*Y + Z*Wd)/2^384 mod p, in [0, 2p), to the stream w; the quotient digits m_i live in
    M(i) and the result limb j overwrites M(j) (m_j is dead from column j + 12 on)."""
    _comba(w, [(X, Y), (Z, Wd)], M, M, 48, ELIDE)


def _gen_prod(w, X, Y, M, R=None):
    """Appends r = X*Y/2^384 mod p, in [0, 2p), to the stream w (gen_mul's column schedule on named registers):
    quotient digits in M(i), result limb j over M(j) or, with R = X, over X(j) (both are dead from column
    j + 12 on)."""
    _comba(w, [(X, Y)], M, R or M, 48, ELIDE)


def _gen_sopn(w, pairs, M):
    """Appends r = (sum of X*Y over `pairs`)/2^384 mod p to the stream w (_gen_sop with any number of product
    terms per column): quotient digits in M(i), result limb j over M(j)."""
    first = [True]
    src2 = ["v[48:49]"]

    def mac(x, y):
        w("v_mad_u64_u32 v[48:49], vcc, %s, %s, %s" % (x, y, src2[0]))
        src2[0] = "v[48:49]"
        if first[0]:
            w("v_addc_co_u32_e64 v51, vcc, 0, 0, vcc")
            first[0] = False
        else:
            w("v_addc_co_u32_e32 v51, vcc, 0, v51, vcc")

    def shift():
        w("v_mov_b32 v50, v49")
        src2[0] = "v[50:51]"
        first[0] = True

    Sp = lambda j: "s%d" % (16 + j)
    X0, Y0 = pairs[0]
    w("v_mad_u64_u32 v[48:49], vcc, %s, %s, 0" % (X0(0), Y0(0)))
    w("v_mov_b32 v51, 0")
    first[0] = False
    for X, Y in pairs[1:]:
        mac(X(0), Y(0))
    w("v_mul_lo_u32 %s, v48, s28" % M(0))
    mac(M(0), "s16")
    shift()
    for i in range(1, N32):
        for j in range(i):
            for X, Y in pairs:
                mac(X(j), Y(i - j))
            mac(M(j), Sp(i - j))
        for X, Y in pairs:
            mac(X(i), Y(0))
        w("v_mul_lo_u32 %s, v48, s28" % M(i))
        mac(M(i), "s16")
        shift()
    for i in range(N32, 2 * N32 - 1):
        for j in range(i - N32 + 1, N32):
            for X, Y in pairs:
                mac(X(j), Y(i - j))
            mac(M(j), Sp(i - j))
        w("v_mov_b32 %s, v48" % M(i - N32))
        shift()
    w("v_mov_b32 %s, v50" % M(N32 - 1))


# EXPERIMENT (lazy reduction): an Fp2 sum of two products with ONE Montgomery reduction per output
# coefficient -- double-width accumulation of four 384 x 384 products per column:
#   c1 = (x0 y1 + x1 y0 + z0 w1 + z1 w0)/R,   c0 = (x0 y0 + x1 (2p - y1) + z0 w0 + z1 (2p - w1))/R
# 2 x 720 mads for x y + z w against 2 x 864 for two gen_fp2_mul calls plus an Fp2 addition.  Canonical operands
# (< p): each sum is < 6p^2 < pR, the output < 1.61p, one conditional subtraction.  Registers: x0 = v[0:11],
# x1 = v[12:23], y0 = v[24:35], y1 = v[36:47], z0 = v[88:99], z1 = v[100:111], w0 = v[112:123], w1 = v[124:135];
# c1 -> v[52:63], c0 -> v[64:75]; y1 and w1 clobbered, v48-v51, v76-v87, s16-s28, vcc clobbered.
FP2M2_Z0, FP2M2_Z1, FP2M2_W0, FP2M2_W1 = 88, 100, 112, 124


# ... and the three-product form (fp12_sqr_l's dense Fp6 products as schoolbook sums): c = x y + z w + u t with
# u0 = v[136:147], u1 = v[148:159], t0 = v[160:171], t1 = v[172:183] (t1 clobbered as well).  Canonical operands: each
# coefficient's sum is < 9p^2 < pR (p < 2^380.8), the output < 1.92p.
FP2M3_U0, FP2M3_U1, FP2M3_T0, FP2M3_T1 = 136, 148, 160, 172


def gen_fp2_mul3():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    P2L = [((2 * P) >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    X0, X1, Y0, Y1, C1, C0, T = V(0), V(12), V(24), V(36), V(FP2_C1), V(FP2_C0), V(FP2_T)
    Z0, Z1, W0, W1 = V(FP2M2_Z0), V(FP2M2_Z1), V(FP2M2_W0), V(FP2M2_W1)
    U0, U1, T0, T1 = V(FP2M3_U0), V(FP2M3_U1), V(FP2M3_T0), V(FP2M3_T1)
    out = []
    w = out.append
    for j in range(N32):
        w("s_mov_b32 s%d, 0x%08x" % (16 + j, PL[j]))
    w("s_mov_b32 s28, 0x%08x" % PINV32)
    _gen_sopn(w, [(X0, Y1), (X1, Y0), (Z0, W1), (Z1, W0), (U0, T1), (U1, T0)], C1)
    for j in range(N32):
        w("v_mov_b32 %s, 0x%08x" % (C0(j), P2L[j]))
    for B in (Y1, W1, T1):
        w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (B(0), C0(0), B(0)))
        for j in range(1, N32):
            w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (B(j), C0(j), B(j)))
    _gen_sopn(w, [(X0, Y0), (X1, Y1), (Z0, W0), (Z1, W1), (U0, T0), (U1, T1)], C0)
    for j in range(N32):
        w("v_mov_b32 %s, s%d" % (Y1(j), 16 + j))
    for C in (C1, C0):
        _final_sub(w, C, Y1, T, "v48")
    return out


def gen_fp2_mul2():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    P2L = [((2 * P) >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    X0, X1, Y0, Y1, C1, C0, T = V(0), V(12), V(24), V(36), V(FP2_C1), V(FP2_C0), V(FP2_T)
    Z0, Z1, W0, W1 = V(FP2M2_Z0), V(FP2M2_Z1), V(FP2M2_W0), V(FP2M2_W1)
    out = []
    w = out.append
    for j in range(N32):
        w("s_mov_b32 s%d, 0x%08x" % (16 + j, PL[j]))
    w("s_mov_b32 s28, 0x%08x" % PINV32)
    _gen_sopn(w, [(X0, Y1), (X1, Y0), (Z0, W1), (Z1, W0)], C1)   # c1 (raw, < 2p)
    for j in range(N32):                                           # 2p into VGPRs
        w("v_mov_b32 %s, 0x%08x" % (C0(j), P2L[j]))
    for B in (Y1, W1):                                             # y1 <- 2p - y1, w1 <- 2p - w1
        w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (B(0), C0(0), B(0)))
        for j in range(1, N32):
            w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (B(j), C0(j), B(j)))
    _gen_sopn(w, [(X0, Y0), (X1, Y1), (Z0, W0), (Z1, W1)], C0)   # c0 (raw)
    for j in range(N32):                                           # p over the dead 2p - y1
        w("v_mov_b32 %s, s%d" % (Y1(j), 16 + j))
    for C in (C1, C0):
        _final_sub(w, C, Y1, T, "v48")
    return out


# Fp2 squaring: c0 = (a0 + a1)(a0 + p - a1)/R, c1 = a0 (a1 + a1)/R.  The three operand sums stay unreduced
# (< 2p each, products < 4p^2 < pR) and the doubling of c1 moves onto an operand, so the routine is two products,
# three 12-word add/sub chains and two final subtractions.  a0 = v[0:11], a1 = v[12:23] (clobbered); c0 -> v[24:35],
# c1 -> v[36:47]; v48-v63, s16-s28, vcc clobbered.
FP2S_A0, FP2S_A1, FP2S_C0, FP2S_C1 = 0, 12, 24, 36


def gen_fp2_sqr():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    A0, A1, C0, C1 = V(FP2S_A0), V(FP2S_A1), V(FP2S_C0), V(FP2S_C1)
    out = []
    w = out.append
    _p_sgprs(w)
    # d = (p - a1) + a0 into C1 (p staged in C0 first), s = a0 + a1 into C0, a1 <- 2 a1
    _load_p(w, C0)
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (C1(0), C0(0), A1(0)))
    for j in range(1, N32):
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (C1(j), C0(j), A1(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (C1(0), C1(0), A0(0)))
    for j in range(1, N32):
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (C1(j), C1(j), A0(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (C0(0), A0(0), A1(0)))
    for j in range(1, N32):
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (C0(j), A0(j), A1(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (A1(0), A1(0), A1(0)))
    for j in range(1, N32):
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (A1(j), A1(j), A1(j)))
    T = V(52)
    _gen_prod(w, C0, C1, T, R=C0)                      # c0 = s d (raw) over s; digits in v52..v63
    _gen_prod(w, A0, A1, C1)                           # c1 = a0 (2 a1) (raw); digits and result over d
    _load_p(w, A0)
    for C in (C0, C1):                                 # canonical: keep c when c - p borrows
        w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (T(0), C(0), A0(0)))
        for j in range(1, N32):
            w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (T(j), C(j), A0(j)))
        for j in range(N32):
            w("v_cndmask_b32_e64 %s, %s, %s, vcc" % (C(j), T(j), C(j)))
    return out


def gen_fp2_mul():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    A0, A1, B0, B1, C1, C0 = (V(FP2_A0), V(FP2_A1), V(FP2_B0), V(FP2_B1), V(FP2_C1), V(FP2_C0))
    out = []
    w = out.append
    _p_sgprs(w)
    P2L = [((2 * P) >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    T = V(FP2_T)
    _gen_sop(w, A0, B1, A1, B0, C1)                    # c1 (raw, < 2p) in v[52:63]
    for j in range(N32):                               # 2p into VGPRs (the carry chain reads vcc: one
        w("v_mov_b32 %s, 0x%08x" % (C0(j), P2L[j]))    # constant-bus operand only)
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (B1(0), C0(0), B1(0)))
    for j in range(1, N32):                            # b1 <- 2p - b1 in (0, 2p]
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (B1(j), C0(j), B1(j)))
    _gen_sop(w, A0, B0, A1, B1, C0)                    # c0 (raw) in v[64:75]
    _load_p(w, B1)                                     # p over the dead 2p - b1; a0, a1, b0 stay intact
    for C in (C1, C0):                                 # canonical: keep c when c - p borrows
        w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (T(0), C(0), B1(0)))
        for j in range(1, N32):
            w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (T(j), C(j), B1(j)))
        for j in range(N32):
            w("v_cndmask_b32_e64 %s, %s, %s, vcc" % (C(j), T(j), C(j)))
    return out


# Lane-pair halves of the Fp2 product and square (the split-Fp2 build, BLS_FP2_PAIR: an Fp2 value is held in full on
# two lanes and each lane computes ONE output coefficient, then the lanes swap; field.h / tower.h).  The lane's half
# arrives as a mask in v76 (0: c0, ~0: c1); the operand choice is a v_bfi_b32 per word, so both lanes run the same
# stream.  Same operand ranges and canonical output as gen_fp2_mul / gen_fp2_sqr.
# Product half: a0 = v[0:11], a1 = v[12:23] (preserved), b0 = v[24:35], b1 = v[36:47] (clobbered); the half
#   c0 = (a0 b0 + a1 (2p - b1))/R or c1 = (a0 b1 + a1 b0)/R -> v[52:63]; v48-v51, v64-v75, s16-s28, vcc clobbered.
# Square half: a0 = v[0:11], a1 = v[12:23] (preserved); c0 = (a0 + a1)(a0 + p - a1)/R or c1 = a0 (2 a1)/R ->
#   v[24:35]; v36-v75, s16-s28, vcc clobbered.
FP2H_MASK, FP2H_OUT, FP2HS_OUT = 76, 52, 24


def _final_sub(w, C, PR, T, mask=None):
    """C <- C - p when that does not borrow (C < 2p -> canonical); PR holds p, T is scratch."""
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (T(0), C(0), PR(0)))
    for j in range(1, N32):
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (T(j), C(j), PR(j)))
    for j in range(N32):  # the borrow selects straight from VCC (the e64 form: one slot, unlike the VOP2 one)
        w("v_cndmask_b32_e64 %s, %s, %s, vcc" % (C(j), T(j), C(j)))


def gen_fp2_mul_half():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    P2L = [((2 * P) >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    A0, A1, B0, B1, C, T = V(0), V(12), V(24), V(36), V(FP2H_OUT), V(64)
    HM = "v%d" % FP2H_MASK
    out = []
    w = out.append
    _p_sgprs(w)
    for j in range(N32):                               # 2p staged in C (one constant-bus operand per carry step)
        w("v_mov_b32 %s, 0x%08x" % (C(j), P2L[j]))
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (T(0), C(0), B1(0)))
    for j in range(1, N32):                            # T <- 2p - b1 in (0, 2p]
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (T(j), C(j), B1(j)))
    for j in range(N32):                               # W = c1 ? b0 : 2p - b1 (over T)
        w("v_bfi_b32 %s, %s, %s, %s" % (T(j), HM, B0(j), T(j)))
    for j in range(N32):                               # Y = c1 ? b1 : b0 (over b1)
        w("v_bfi_b32 %s, %s, %s, %s" % (B1(j), HM, B1(j), B0(j)))
    _gen_sop(w, A0, B1, A1, T, C)                      # (a0 Y + a1 W)/R, raw (< 2p), over C
    _load_p(w, B0)                                     # p over the dead b0
    _final_sub(w, C, B0, T, "v48")
    return out


def gen_fp2_sqr_half():
    PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)
    PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]
    V = lambda base: (lambda j: "v%d" % (base + j))
    A0, A1, X, Y, M, T = V(0), V(12), V(FP2HS_OUT), V(36), V(52), V(64)
    HM = "v%d" % FP2H_MASK
    out = []
    w = out.append
    _p_sgprs(w)
    _load_p(w, X)                                      # p staged in X
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (Y(0), X(0), A1(0)))
    for j in range(1, N32):                            # Y <- p - a1
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (Y(j), X(j), A1(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (Y(0), Y(0), A0(0)))
    for j in range(1, N32):                            # Y <- a0 + p - a1 (d)
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (Y(j), Y(j), A0(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (X(0), A0(0), A1(0)))
    for j in range(1, N32):                            # X <- a0 + a1 (s)
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (X(j), A0(j), A1(j)))
    w("v_add_co_u32_e32 %s, vcc, %s, %s" % (T(0), A1(0), A1(0)))
    for j in range(1, N32):                            # T <- 2 a1
        w("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc" % (T(j), A1(j), A1(j)))
    for j in range(N32):                               # X = c1 ? a0 : s,  Y = c1 ? 2 a1 : d
        w("v_bfi_b32 %s, %s, %s, %s" % (X(j), HM, A0(j), X(j)))
        w("v_bfi_b32 %s, %s, %s, %s" % (Y(j), HM, T(j), Y(j)))
    _gen_prod(w, X, Y, M, R=X)                         # X Y / R, raw (< 2p), over X
    _load_p(w, T)                                      # p for the final subtraction
    _final_sub(w, X, T, M, "v48")
    return out


# ---------------------------------------------------------------- modular add / sub / neg
# One asm block each, operands allocated by the compiler (positional: outputs r = %0-%11, t = %12-%23,
# m = %24; inputs a = %25-%36, then b = %37-%48 and p = %49-%60, or p = %37-%48 for neg).  One VCC carry chain
# per block: compiled C++ interleaves the chains of independent adds on VCC and an SGPR pair, which costs an
# s_nop per step (VALU-written carry read back two instructions later), and selects with the VOP2
# v_cndmask_b32_e32 (~19 cycles on gfx950).  Here the borrow becomes a lane mask m = -borrow in a VGPR
# (v_subb_co_u32_e64 m, vcc, 0, 0, vcc) and the select is v_bfi_b32 / v_and_b32.  p must sit in VGPRs: a
# carry-in VCC plus a literal or SGPR operand exceeds the gfx9 constant-bus limit of one.
def gen_add():
    """r = a + b mod p for a, b < p: s = a + b, d = s - p, keep s when d borrows."""
    w = []
    w.append("v_add_co_u32_e32 %0, vcc, %25, %37")
    for i in range(1, 12):
        w.append("v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 25 + i, 37 + i))
    w.append("v_sub_co_u32_e32 %12, vcc, %0, %49")
    for i in range(1, 12):
        w.append("v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (12 + i, i, 49 + i))
    for i in range(12):  # keep s where s - p borrows (VCC), else s - p; %24 is left unused
        w.append("v_cndmask_b32_e64 %%%d, %%%d, %%%d, vcc" % (i, 12 + i, i))
    return w


def gen_sub(neg=False):
    """r = a - b mod p (neg: r = 0 - a): d = a - b, then d + (p & -borrow)."""
    pb = 37 if neg else 49
    w = []
    if neg:
        w.append("v_sub_co_u32_e32 %0, vcc, 0, %25")
        for i in range(1, 12):
            w.append("v_subb_co_u32_e32 %%%d, vcc, 0, %%%d, vcc" % (i, 25 + i))
    else:
        w.append("v_sub_co_u32_e32 %0, vcc, %25, %37")
        for i in range(1, 12):
            w.append("v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 25 + i, 37 + i))
    for i in range(12):  # p where a - b borrowed (VCC), else 0; %24 is left unused
        w.append("v_cndmask_b32_e64 %%%d, 0, %%%d, vcc" % (12 + i, pb + i))
    w.append("v_add_co_u32_e32 %0, vcc, %0, %12")
    for i in range(1, 12):
        w.append("v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, i, 12 + i))
    return w


def gen_add_lazy():
    """r = a + b WITHOUT reduction (a, b < p -> r < 2p): only ever a product operand.  The product reduces any
    operands with a*b < p*2^384, which 2p*2p satisfies (4p < 2^384).  Operands: r = %0-%11, a = %12-%23,
    b = %24-%35."""
    w = ["v_add_co_u32_e32 %0, vcc, %12, %24"]
    for i in range(1, 12):
        w.append("v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 12 + i, 24 + i))
    return w


def gen_sub_lazy():
    """r = a + (p - b) WITHOUT reduction (a, b < p -> 0 < r < 2p): a product operand standing for a - b.
    Operands: r = %0-%11, t = %12-%23 (p - b), a = %24-%35, b = %36-%47, p = %48-%59."""
    w = ["v_sub_co_u32_e32 %12, vcc, %48, %36"]
    for i in range(1, 12):
        w.append("v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (12 + i, 48 + i, 36 + i))
    w.append("v_add_co_u32_e32 %0, vcc, %24, %12")
    for i in range(1, 12):
        w.append("v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 24 + i, 12 + i))
    return w


def emulate_positional(body, outs, ins):
    """Interprets an add/sub/neg block: ins = list of input values by operand number (25..)."""
    reg = {}
    for k, v in ins.items():
        reg[k] = v
    s = {"vcc": 0}
    M32 = 0xFFFFFFFF

    def rd(x):
        x = x.strip()
        if x == "vcc":
            return s["vcc"]
        if x.startswith("%"):
            return reg[int(x[1:])]
        return int(x, 0)

    for ins_ in body:
        op, rest = ins_.split(" ", 1)
        o = [t.strip() for t in rest.split(",")]
        d = int(o[0][1:])
        if op == "v_add_co_u32_e32":
            r = rd(o[2]) + rd(o[3])
            reg[d], s["vcc"] = r & M32, r >> 32
        elif op == "v_addc_co_u32_e32":
            r = rd(o[2]) + rd(o[3]) + rd(o[4])
            reg[d], s["vcc"] = r & M32, r >> 32
        elif op == "v_sub_co_u32_e32":
            r = rd(o[2]) - rd(o[3])
            reg[d], s["vcc"] = r & M32, 1 if r < 0 else 0
        elif op in ("v_subb_co_u32_e32", "v_subb_co_u32_e64"):
            r = rd(o[2]) - rd(o[3]) - rd(o[4])
            reg[d], s["vcc"] = r & M32, 1 if r < 0 else 0
        elif op == "v_bfi_b32":
            m = rd(o[1])
            reg[d] = (m & rd(o[2])) | (~m & M32 & rd(o[3]))
        elif op == "v_and_b32_e32":
            reg[d] = rd(o[1]) & rd(o[2])
        elif op == "v_cndmask_b32_e64":
            reg[d] = rd(o[2]) if rd(o[3]) else rd(o[1])
        else:
            raise ValueError(ins_)
    return [reg[k] for k in outs]


# ---------------------------------------------------------------- CPU interpreter
class DroppedCarry(AssertionError):
    pass


def emulate(body, a, b, regs=None, strict=True):
    """Interprets the instruction subset used above (one lane); a, b: 12 x 32-bit limbs.
    Returns the 12 output limbs (v0..v11).  With regs (a dict VGPR number -> value, updated in place)
    the register file starts from regs instead of a in v0.. and b in v12..  strict: a v_mad_u64_u32 whose
    carry-out is set must be followed by the v_addc that catches it (carry elision, _comba), else DroppedCarry."""
    v, s = ({}, {}) if regs is None else (regs, {})
    for j in range(N32):  # the callers' SGPRs (P_SGPR): p and -p^-1 mod 2^32
        s["s%d" % (16 + j)] = PL32[j]
    s["s28"] = (-pow(P, -1, 1 << 32)) % (1 << 32)
    pending = [None]
    M32, M64 = 0xFFFFFFFF, (1 << 64) - 1
    if regs is None:
        for j in range(N32):
            v[j], v[12 + j] = a[j], b[j]

    def rd(x):
        x = x.strip()
        if x.startswith("0x"):
            return int(x, 16)
        if x.lstrip("-").isdigit():
            return int(x)
        if x == "vcc":
            return s.get("vcc", 0)
        if x.startswith("v["):
            lo = int(x[2:x.index(":")])
            return v[lo] | (v[lo + 1] << 32)
        if x.startswith("s["):
            lo = int(x[2:x.index(":")])
            return s["s%d" % lo] | (s["s%d" % (lo + 1)] << 32)
        if x.startswith("s"):
            return s[x]
        return v[int(x[1:])]

    def wr(x, val):
        x = x.strip()
        if x.startswith("v["):
            lo = int(x[2:x.index(":")])
            v[lo], v[lo + 1] = val & M32, (val >> 32) & M32
        elif x.startswith("s") or x == "vcc":
            s[x] = val
        else:
            v[int(x[1:])] = val & M32

    for ins in body:
        op, rest = ins.split(" ", 1)
        o = [t.strip() for t in rest.split(",")]
        if pending[0] is not None:
            if strict and not (op.startswith("v_addc_co_u32") and o[-1] == "vcc"):
                raise DroppedCarry(pending[0])
            pending[0] = None
        if op == "s_mov_b32":
            s[o[0]] = rd(o[1])
        elif op in ("v_mov_b32", "v_mov_b64"):
            wr(o[0], rd(o[1]))
        elif op == "v_mad_u64_u32":
            r = (rd(o[2]) & M32) * (rd(o[3]) & M32) + rd(o[4])
            wr(o[0], r & M64)
            s[o[1]] = r >> 64
            if r >> 64:
                pending[0] = ins
        elif op == "v_mul_lo_u32":
            wr(o[0], rd(o[1]) * rd(o[2]))
        elif op.startswith("v_addc_co_u32"):
            r = rd(o[2]) + rd(o[3]) + rd(o[4])
            wr(o[0], r)
            s["vcc"] = r >> 32
        elif op == "v_add_co_u32_e32":
            r = rd(o[2]) + rd(o[3])
            wr(o[0], r)
            s["vcc"] = r >> 32
        elif op == "v_sub_co_u32_e32":
            r = rd(o[2]) - rd(o[3])
            wr(o[0], r)
            s["vcc"] = 1 if r < 0 else 0
        elif op in ("v_subb_co_u32_e32", "v_subb_co_u32_e64"):
            r = rd(o[2]) - rd(o[3]) - rd(o[4])
            wr(o[0], r)
            s["vcc"] = 1 if r < 0 else 0
        elif op == "v_bfi_b32":
            m = rd(o[1])
            wr(o[0], (m & rd(o[2])) | (~m & M32 & rd(o[3])))
        elif op in ("v_cndmask_b32_e32", "v_cndmask_b32_e64"):
            wr(o[0], rd(o[2]) if rd(o[3]) else rd(o[1]))
        elif op == "v_lshrrev_b32":
            wr(o[0], rd(o[2]) >> rd(o[1]))
        elif op == "v_lshrrev_b64":
            wr(o[0], rd(o[2]) >> rd(o[1]))
        elif op == "v_bfe_u32":
            wr(o[0], (rd(o[1]) >> rd(o[2])) & ((1 << rd(o[3])) - 1))
        elif op == "v_alignbit_b32":
            wr(o[0], (((rd(o[1]) << 32) | rd(o[2])) >> rd(o[3])) & M32)
        elif op == "v_and_b32_e32":
            wr(o[0], rd(o[1]) & rd(o[2]))
        elif op == "v_lshl_or_b32":
            wr(o[0], ((rd(o[1]) << rd(o[2])) | rd(o[3])) & M32)
        elif op == "v_lshl_add_u64":
            wr(o[0], ((rd(o[1]) << rd(o[2])) + rd(o[3])) & M64)
        else:
            raise ValueError(ins)
    if strict and pending[0] is not None:
        raise DroppedCarry(pending[0])
    return [v[j] for j in range(N32)]


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(N32)]


def value(l):
    return sum(x << (32 * i) for i, x in enumerate(l))


def check(body, square=False, trials=300, seed=1, mont=R_MONT, canonical=False):
    """Host check of an emitted body: result == a*b/mont mod p, < 2p (or < p when canonical), for inputs
    < 2^384 (< p for the canonical radix-2^32 routine)."""
    rng = random.Random(seed)
    rinv = pow(mont, -1, P)
    edge = [0, 1, P - 1, P, 2 * P - 1, (1 << 384) - 1, (1 << 383), P + 1]
    for t in range(trials):
        if t < len(edge) ** 2:
            a, b = edge[t % len(edge)], edge[t // len(edge) % len(edge)]
        else:
            a, b = rng.randrange(1 << 384), rng.randrange(1 << 384)
        if canonical:
            a, b = a % P, b % P
        if square:
            b = a
        got = value(emulate(body, limbs(a), limbs(b)))
        want = a * b * rinv % P
        assert got < (P if canonical else 2 * P), (hex(a), hex(b), hex(got))
        assert got % P == want, (hex(a), hex(b))
    return True


def body_text(square=False, chains=2, sched=True, pool=("vcc",)):
    SDST_POOL[:] = list(pool)
    _sdst_next[0] = 0
    ins = gen_mul29(square=square, chains=chains)
    if not sched:
        return [x.text for x in ins], 0
    order, cyc = schedule(ins)
    return [x.text for x in order], cyc


def emit_header(path, bodies, extra=()):
    lines = ["// GENERATED by charon_amd/tools/gen_fp_asm.py -- do not edit.",
             "// gfx950 Montgomery product r = a*b/2^384 mod p (canonical), product scanning, %d instructions."
             % len(bodies[0][1]),
             "#pragma once"]
    for name, body in bodies:
        lines.append("// %s: %d instructions" % (name, len(body)))
        lines.append("#define %s \\" % name)
        for k, ins in enumerate(body):
            sep = "\\n\\t" if k + 1 < len(body) else ""
            lines.append('  "%s%s" \\' % (ins, sep))
        lines.append("")
    sg = "" if P_SGPR else ", " + ", ".join('"s%d"' % r for r in range(16, 29))  # s16-s28: inputs with P_SGPR
    clob = ", ".join('"v%d"' % r for r in range(24, 40)) + ', "vcc"' + sg
    lines.append("#define BLS_FP_MUL_ASM_CLOBBERS %s" % clob)
    clob2 = ", ".join('"v%d"' % r for r in list(range(48, 52)) + list(range(76, 88))) + ', "vcc"' + sg
    lines.append("#define BLS_FP2_MUL_ASM_CLOBBERS %s" % clob2)
    clob3 = ", ".join('"v%d"' % r for r in range(48, 64)) + ', "vcc"' + sg
    lines.append("#define BLS_FP2_SQR_ASM_CLOBBERS %s" % clob3)
    clob4 = ", ".join('"v%d"' % r for r in list(range(48, 52)) + list(range(64, 76))) + ', "vcc"' + sg
    lines.append("#define BLS_FP2_MUL_HALF_ASM_CLOBBERS %s" % clob4)
    clob5 = ", ".join('"v%d"' % r for r in range(36, 76)) + ', "vcc"' + sg
    lines.append("#define BLS_FP2_SQR_HALF_ASM_CLOBBERS %s" % clob5)
    for name, body in extra:
        lines.append("")
        lines.append("// %s: %d instructions, positional operands (see tools/gen_fp_asm.py)" % (name, len(body)))
        lines.append("#define %s \\" % name)
        for k, ins in enumerate(body):
            sep = "\\n\\t" if k + 1 < len(body) else ""
            lines.append('  "%s%s" \\' % (ins, sep))
        lines.append("")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def emit_lazy_header(path):
    """The lazy-reduction experiment's routines (gen_fp2_mul2 / gen_fp2_mul3; VERDICT r04 item 7, measured -1.8 % in
    round 5 and off): ~7,300 lines that only a BLS_LAZY_FP6=1 build reads, so they are generated on demand
    (`gen_fp_asm.py --lazy`) instead of shipping in the product header."""
    lines = ["// GENERATED by charon_amd/tools/gen_fp_asm.py --lazy -- do not edit (BLS_LAZY_FP6=1 builds only).",
             "#pragma once"]
    for name, body in (("BLS_FP2_MUL2_ASM_BODY", gen_fp2_mul2()), ("BLS_FP2_MUL3_ASM_BODY", gen_fp2_mul3())):
        lines.append("// %s: %d instructions" % (name, len(body)))
        lines.append("#define %s \\" % name)
        for k, ins in enumerate(body):
            sep = "\\n\\t" if k + 1 < len(body) else ""
            lines.append('  "%s%s" \\' % (ins, sep))
        lines.append("")
    clob6 = ", ".join('"v%d"' % r for r in list(range(48, 52)) + list(range(76, 88))) + ', "vcc", ' + \
        ", ".join('"s%d"' % r for r in range(16, 29))
    lines.append("#define BLS_FP2_MUL2_ASM_CLOBBERS %s" % clob6)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main(lazy=False):
    mul = gen_mul()
    check(mul, mont=1 << 384, canonical=True)
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(pkg, "csrc", "fp_asm_gfx950.h")
    fp2 = gen_fp2_mul()
    fp2s = gen_fp2_sqr()
    emit_header(path, [("BLS_FP_MUL_ASM_BODY", mul), ("BLS_FP2_MUL_ASM_BODY", fp2), ("BLS_FP2_SQR_ASM_BODY", fp2s),
                       ("BLS_FP2_MUL_HALF_ASM_BODY", gen_fp2_mul_half()),
                       ("BLS_FP2_SQR_HALF_ASM_BODY", gen_fp2_sqr_half())],
                extra=[("BLS_FP_ADD_ASM", gen_add()), ("BLS_FP_SUB_ASM", gen_sub()), ("BLS_FP_NEG_ASM", gen_sub(neg=True)),
                       ("BLS_FP_ADD_LAZY_ASM", gen_add_lazy()), ("BLS_FP_SUB_LAZY_ASM", gen_sub_lazy())])
    print("wrote %s: %d instructions" % (path, len(mul)))
    if lazy:
        lpath = os.path.join(pkg, "tools", "fp_asm_lazy_gfx950.h")
        emit_lazy_header(lpath)
        print("wrote %s" % lpath)


if __name__ == "__main__":
    import sys
    main(lazy="--lazy" in sys.argv)
