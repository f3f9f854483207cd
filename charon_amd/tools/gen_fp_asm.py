"""Generate charon_amd/csrc/fp_asm_gfx950.h: the gfx950 Montgomery product as one inline-asm block.

Why asm: hipcc cannot fuse the carry-out of v_mad_u64_u32 into the next add, so compiled C++
spends ~4 instructions per 32x32 limb product.  Here every product is exactly
    v_mad_u64_u32 acc, vcc, x, y, acc      (64-bit accumulate, carry-out -> vcc)
    v_addc_co_u32 t, vcc, 0, t, vcc        (carry -> third accumulator word)
in product-scanning (Comba) order with the Montgomery reduction interleaved per column
(Koc-Acar-Kaliski "FIPS").  Registers are pinned (a = v[0:11] in/out, b = v[12:23]) to match the
AMDGPU calling convention of a non-inlined function taking/returning 12-dword vectors, so a call
costs no moves.  Only caller-saved registers are used (v0-v39, vcc, s16-s28).

Correctness is covered by the GPU parity tests (every curve/pairing result goes through it); the
host build keeps the C++ CIOS in field.h, which the CPU tests diff against the oracle.

Run:  python3 charon_amd/tools/gen_fp_asm.py
"""
import os

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
N = 12
PINV = (-pow(P, -1, 1 << 32)) % (1 << 32)
PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N)]

A = lambda j: "v%d" % j          # a limbs, later the output
B = lambda j: "v%d" % (12 + j)   # b limbs, later the subtraction temp
M = lambda j: "v%d" % (24 + j)   # Montgomery quotients
ACC = "v[36:37]"
ACC_LO, ACC_HI = "v36", "v37"
T = "v39"                        # carry word; v38 takes the old hi at a column shift, so that
SHIFTED, SHIFTED_LO = "v[38:39]", "v38"  # (old hi, T) is an aligned pair the next mad reads
SP = lambda j: "s%d" % (16 + j)  # p limbs
SPINV = "s28"


def gen_mul(square=False):
    out = []
    w = out.append
    for j in range(N):
        w("s_mov_b32 %s, 0x%08x" % (SP(j), PL[j]))
    w("s_mov_b32 %s, 0x%08x" % (SPINV, PINV))
    first_in_col = [True]
    src2 = [ACC]

    def mac(x, y):
        w("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (ACC, x, y, src2[0]))
        src2[0] = ACC
        if first_in_col[0]:
            w("v_addc_co_u32_e64 %s, vcc, 0, 0, vcc" % T)
            first_in_col[0] = False
        else:
            w("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (T, T))

    def shift():
        # one move, not two: the next column's first mad reads (old hi, T) as v[38:39] and writes
        # the fresh accumulator v[36:37] (64-bit VGPR operands must be even-aligned on gfx950)
        w("v_mov_b32 %s, %s" % (SHIFTED_LO, ACC_HI))
        src2[0] = SHIFTED
        first_in_col[0] = True

    # column 0: acc = a0*b0 (no carry possible)
    w("v_mad_u64_u32 %s, vcc, %s, %s, 0" % (ACC, A(0), B(0)))
    w("v_mov_b32 %s, 0" % T)
    first_in_col[0] = False
    w("v_mul_lo_u32 %s, %s, %s" % (M(0), ACC_LO, SPINV))
    mac(M(0), SP(0))
    shift()
    for i in range(1, N):
        for j in range(i):
            mac(A(j), B(i - j))
            mac(M(j), SP(i - j))
        mac(A(i), B(0))
        w("v_mul_lo_u32 %s, %s, %s" % (M(i), ACC_LO, SPINV))
        mac(M(i), SP(0))
        shift()
    for i in range(N, 2 * N - 1):
        for j in range(i - N + 1, N):
            mac(A(j), B(i - j))
            mac(M(j), SP(i - j))
        w("v_mov_b32 %s, %s" % (A(i - N), ACC_LO))  # a[i-12] is dead from column i on
        shift()
    w("v_mov_b32 %s, %s" % (A(N - 1), SHIFTED_LO))
    # conditional subtraction: d = o - p into b's registers; keep o when it borrows.  p is copied
    # to the (dead) quotient registers first: a carry-in vcc plus an SGPR operand would exceed the
    # gfx9 constant-bus limit of one scalar read per VALU instruction.
    for j in range(N):
        w("v_mov_b32 %s, %s" % (M(j), SP(j)))
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (B(0), A(0), M(0)))
    for j in range(1, N):
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (B(j), A(j), M(j)))
    for j in range(N):
        w("v_cndmask_b32_e32 %s, %s, %s, vcc" % (A(j), B(j), A(j)))
    return out


# --- two-chain product (experiment, NOT emitted) ----------------------------------------------
# Measured on MI355X (profiles/r01_fp_product_experiments.txt): bit-exact, but C2 fell from 917k
# to 841k verifies/s.  The single chain is already ~80 % instruction-issue bound (695 VALU
# instructions x 4 cycles per wave64 = 2,780 of the ~3,500 cycles a product takes at one wave per
# SIMD), so the 92 extra instructions cost more than the hidden carry latency saves.  Kept as the
# record of the experiment; the hypothesis it tested was:
# the single-chain form above is latency-bound at one wave per SIMD: every v_mad_u64_u32 reads
# the previous one's accumulator and every v_addc_co_u32 waits ~20 cycles for the carry the mad
# just wrote to vcc (profiles/r01_lat_probe.txt: 24.8 cycles per mad+addc pair).  Here
#   * the a*b terms (chain X) and the m*p terms (chain Y) of a column accumulate independently and
#     are interleaved, so each mad's accumulator dependency is two instructions back;
#   * every mad writes its carry to the next SGPR pair of a rotating pool and the addc that
#     consumes it is issued DEFER instructions later, when the carry has landed;
#   * the columns meet once: Y += lo(X) (a mad by 1), then m_i = lo(Y)*p' and Y += m_i*p0 zeroes
#     the column (i < 12) or lo(Y) is output word i-12 (i >= 12).
# The sum X+Y is the same 768-bit value the single chain builds, so results are bit-identical.
XACC, XL, XH, XT = "v[36:37]", "v36", "v37", "v38"
YACC, YL, YH, YT = "v[40:41]", "v40", "v41", "v39"
CARRY_POOL = ["vcc"] + ["s[%d:%d]" % (r, r + 1) for r in range(40, 54, 2)]
DEFER = 3


def gen_mul2(defer=DEFER):
    out = []
    w = out.append
    for j in range(N):
        w("s_mov_b32 %s, 0x%08x" % (SP(j), PL[j]))
    w("s_mov_b32 %s, 0x%08x" % (SPINV, PINV))
    pool = list(CARRY_POOL)
    nxt = [0]
    pending = []          # (T register, carry pair, first-in-column)
    t_init = {XT: False, YT: False}

    def take():
        c = pool[nxt[0] % len(pool)]
        nxt[0] += 1
        assert all(c != p[1] for p in pending), "carry pool too small for DEFER"
        return c

    def emit_addc():
        t, c, first = pending.pop(0)
        src = "0" if first else t
        if c == "vcc":
            if first:
                w("v_addc_co_u32_e64 %s, vcc, 0, 0, vcc" % t)
            else:
                w("v_addc_co_u32_e32 %s, vcc, 0, %s, vcc" % (t, t))
        else:
            w("v_addc_co_u32_e64 %s, %s, 0, %s, %s" % (t, c, src, c))

    def mad(acc, t, x, y):
        c = take()
        w("v_mad_u64_u32 %s, %s, %s, %s, %s" % (acc, c, x, y, acc))
        first = not t_init[t]
        t_init[t] = True
        pending.append((t, c, first))
        while len(pending) > defer:
            emit_addc()

    def flush():
        while pending:
            emit_addc()

    def shift():
        for lo, hi, t in ((XL, XH, XT), (YL, YH, YT)):
            if t_init[t]:
                w("v_mov_b32 %s, %s" % (lo, hi))
                w("v_mov_b32 %s, %s" % (hi, t))
            else:
                w("v_mov_b32 %s, %s" % (lo, hi))
                w("v_mov_b32 %s, 0" % hi)
            t_init[t] = False

    # column 0 seeds both accumulators without reading them
    w("v_mad_u64_u32 %s, vcc, %s, %s, 0" % (XACC, A(0), B(0)))
    w("v_mul_lo_u32 %s, %s, %s" % (M(0), XL, SPINV))
    w("v_mad_u64_u32 %s, vcc, %s, %s, 0" % (YACC, M(0), SP(0)))
    # lo(X)+lo(Y) == 0 mod 2^32; the column carries 1 iff lo(X) != 0.  Fold it as Y += lo(X).
    w("v_mov_b32 %s, 0" % XT)
    w("v_mov_b32 %s, 0" % YT)
    t_init[XT] = t_init[YT] = True
    mad(YACC, YT, XL, "1")
    flush()
    shift()
    for i in range(1, 2 * N - 1):
        xs = [(A(j), B(i - j)) for j in range(max(0, i - N + 1), min(i, N - 1) + 1)]
        ys = [(M(j), SP(i - j)) for j in range(max(0, i - N + 1), min(i, N))]
        for k in range(max(len(xs), len(ys))):
            if k < len(xs):
                mad(XACC, XT, *xs[k])
            if k < len(ys):
                mad(YACC, YT, *ys[k])
        mad(YACC, YT, XL, "1")
        if i < N:
            flush()  # lo(Y) must be final before the quotient is taken
            w("v_mul_lo_u32 %s, %s, %s" % (M(i), YL, SPINV))
            mad(YACC, YT, M(i), SP(0))
        else:
            w("v_mov_b32 %s, %s" % (A(i - N), YL))  # a[i-12] is dead from column i on
        flush()
        shift()
    w("v_add_u32_e32 %s, %s, %s" % (A(N - 1), XL, YL))
    for j in range(N):
        w("v_mov_b32 %s, %s" % (M(j), SP(j)))
    w("v_sub_co_u32_e32 %s, vcc, %s, %s" % (B(0), A(0), M(0)))
    for j in range(1, N):
        w("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc" % (B(j), A(j), M(j)))
    for j in range(N):
        w("v_cndmask_b32_e32 %s, %s, %s, vcc" % (A(j), B(j), A(j)))
    return out


def emulate(body, a, b):
    """Tiny interpreter for the instruction subset above (lane-scalar), used to check the
    generator on the host: returns the 12 output limbs for 12-limb inputs a, b."""
    v, s = {}, {}
    for j in range(N):
        v[j], v[12 + j] = a[j], b[j]
    M32 = 0xFFFFFFFF

    def rd(x):
        if x.startswith("0x"):
            return int(x, 16)
        if x.isdigit():
            return int(x)
        if x.startswith("s["):
            return s[x]
        if x.startswith("s"):
            return s[x]
        if x == "vcc":
            return s["vcc"]
        if x.startswith("v["):
            lo = int(x[2:x.index(":")])
            return v[lo] | (v[lo + 1] << 32)
        return v[int(x[1:])]

    def wr64(x, val):
        lo = int(x[2:x.index(":")])
        v[lo], v[lo + 1] = val & M32, (val >> 32) & M32

    for ins in body:
        op, rest = ins.split(" ", 1)
        ops = [o.strip() for o in rest.split(",")]
        if op == "s_mov_b32":
            s[ops[0]] = rd(ops[1])
        elif op == "v_mov_b32":
            v[int(ops[0][1:])] = rd(ops[1]) & M32
        elif op == "v_mad_u64_u32":
            r = rd(ops[2]) * rd(ops[3]) + rd(ops[4])
            wr64(ops[0], r)
            s[ops[1]] = r >> 64
        elif op == "v_mul_lo_u32":
            v[int(ops[0][1:])] = (rd(ops[1]) * rd(ops[2])) & M32
        elif op.startswith("v_addc_co_u32"):
            r = rd(ops[2]) + rd(ops[3]) + rd(ops[4])
            v[int(ops[0][1:])] = r & M32
            s[ops[1]] = r >> 32
        elif op == "v_add_u32_e32":
            v[int(ops[0][1:])] = (rd(ops[1]) + rd(ops[2])) & M32
        elif op == "v_sub_co_u32_e32":
            r = rd(ops[2]) - rd(ops[3])
            v[int(ops[0][1:])] = r & M32
            s["vcc"] = 1 if r < 0 else 0
        elif op == "v_subb_co_u32_e32":
            r = rd(ops[2]) - rd(ops[3]) - rd(ops[4])
            v[int(ops[0][1:])] = r & M32
            s["vcc"] = 1 if r < 0 else 0
        elif op == "v_cndmask_b32_e32":
            v[int(ops[0][1:])] = rd(ops[2]) if rd(ops[3]) else rd(ops[1])
        else:
            raise ValueError(ins)
    return [v[j] for j in range(N)]


def main():
    body = gen_mul()
    clob = ", ".join('"v%d"' % r for r in range(24, 40)) + ', "vcc", ' + ", ".join('"s%d"' % r for r in range(16, 29))
    lines = []
    lines.append("// GENERATED by charon_amd/tools/gen_fp_asm.py -- do not edit.")
    lines.append("// gfx950 Montgomery product r = a*b/2^384 mod p, product scanning, %d instructions." % len(body))
    lines.append("#pragma once")
    lines.append("#define BLS_FP_MUL_ASM_BODY \\")
    for k, ins in enumerate(body):
        sep = "\\n\\t" if k + 1 < len(body) else ""
        lines.append('  "%s%s" \\' % (ins, sep))
    lines.append("")
    lines.append("#define BLS_FP_MUL_ASM_CLOBBERS %s" % clob)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "fp_asm_gfx950.h")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote", path, len(body), "instructions")


if __name__ == "__main__":
    main()
