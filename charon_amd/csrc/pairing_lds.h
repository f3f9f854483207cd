// The 2-pair Miller loop with its Fp12 accumulator f resident in LDS (k_verify_fused, the C2 kernel).
//
// Why: one Verify lane runs at one wave per SIMD with 512 registers, and the live set of a Miller iteration -- f (144
// dwords), T0/T1 (144), P0/P1 (48), the six line coefficients (72), the doubling temporaries (~120) and the pinned
// operand registers of the asm Fp2 products (88) -- is larger than that, so the iteration went through scratch (441
// dwordx4 loads + 316 stores per doubling iteration).  f is the one large value that is only
// touched coefficient by coefficient, so it lives in LDS instead: 576 B per lane, 36 KiB per 64-lane workgroup,
// 144 KiB for the four one-wave workgroups of a CU (of 160 KiB).  Every Fp2 coefficient is fetched right before the
// product that reads it (3 + 3 ds_read_b128, against the 1,300-instruction Fp2 product) and the squaring and line
// product are reordered so their intermediates overwrite the coefficients they no longer need.
//
// Layout: 16-byte group g (0..35) of lane l at byte 16 (g S + l), S = the workgroup's lane count.  A wave's
// ds_read_b128 of one group then covers 1 KiB of consecutive bytes: conflict-free (MI355X_MICROARCH.md, LDS).  Fp12
// coefficient k (0..5 = c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2) is groups 6k..6k+5 (c0 limbs, then c1 limbs).
//
// The values are the ones pairing.h computes: the same Montgomery operations on the same canonical inputs, in an order
// that only changes which temporaries hold them (tests/test_host_arith.py compares f and the statuses on the host).
#pragma once
#include "pairing.h"

namespace bls {

#if defined(__HIP_DEVICE_COMPILE__)
#define BLS_LDS __attribute__((address_space(3)))
#else
#define BLS_LDS
#endif

typedef uint32_t u32x4 __attribute__((vector_size(16)));  // one ds_read_b128 / ds_write_b128

#if defined(__HIPCC__)
#define BLS_MEMBER __forceinline__
#else
#define BLS_MEMBER inline
#endif

template <int S>
struct f12l {
  BLS_LDS u32x4* p;  // this lane's group 0

  BLS_HD BLS_MEMBER void ld_fp(fp& r, int g) const {
    for (int j = 0; j < 3; ++j) {
      const u32x4 q = p[(g + j) * S];
      r.v[4 * j] = q[0];
      r.v[4 * j + 1] = q[1];
      r.v[4 * j + 2] = q[2];
      r.v[4 * j + 3] = q[3];
    }
  }
  BLS_HD BLS_MEMBER void st_fp(int g, const fp& a) const {
    for (int j = 0; j < 3; ++j) {
      const u32x4 q = {a.v[4 * j], a.v[4 * j + 1], a.v[4 * j + 2], a.v[4 * j + 3]};
      p[(g + j) * S] = q;
    }
  }
  BLS_HD BLS_MEMBER fp2 ld(int k) const {
    fp2 r;
    ld_fp(r.c0, 6 * k);
    ld_fp(r.c1, 6 * k + 3);
    return r;
  }
  BLS_HD BLS_MEMBER void st(int k, const fp2& a) const {
    st_fp(6 * k, a.c0);
    st_fp(6 * k + 3, a.c1);
  }
  BLS_HD BLS_MEMBER void ld12(fp12& r) const {
    r.c0.c0 = ld(0);
    r.c0.c1 = ld(1);
    r.c0.c2 = ld(2);
    r.c1.c0 = ld(3);
    r.c1.c1 = ld(4);
    r.c1.c2 = ld(5);
  }
  BLS_HD BLS_MEMBER void st12(const fp12& a) const {
    st(0, a.c0.c0);
    st(1, a.c0.c1);
    st(2, a.c0.c2);
    st(3, a.c1.c0);
    st(4, a.c1.c1);
    st(5, a.c1.c2);
  }
};

// fp6_mul (tower.h) with the operands' coefficients fetched at each use: a(i), b(i) return coefficient i.
#if BLS_LAZY_FP6
// The lazy-reduction experiment: schoolbook, each output coefficient one sum of three Fp2
// products with ONE Montgomery reduction per Fp coefficient (fp2_mul3): c0 = a0 b0 + (xi a1) b2 + (xi a2) b1,
// c1 = a0 b1 + a1 b0 + (xi a2) b2, c2 = a0 b2 + a1 b1 + a2 b0.  Operands canonical.
template <class A, class B>
BLS_HD BLS_INLINE void fp6_mul_fetch(fp6& r, const A& a, const B& b) {
  fp2 xa1, xa2, c0, c1, c2;
  fp2_mul_xi(xa1, a(1));
  fp2_mul_xi(xa2, a(2));
  fp2_mul3(c0, a(0), b(0), xa1, b(2), xa2, b(1));
  fp2_mul3(c1, a(0), b(1), a(1), b(0), xa2, b(2));
  fp2_mul3(c2, a(0), b(2), a(1), b(1), a(2), b(0));
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
#else
template <class A, class B>
BLS_HD BLS_INLINE void fp6_mul_fetch(fp6& r, const A& a, const B& b) {
  fp2 t0, t1, t2, s0, s1, u0, u1, u2;
  fp2_mul(t0, a(0), b(0));
  fp2_mul(t1, a(1), b(1));
  fp2_mul(t2, a(2), b(2));
  fp2_add_lazy(s0, a(1), a(2));
  fp2_add_lazy(s1, b(1), b(2));
  fp2_mul(u0, s0, s1);
  fp2_sub(u0, u0, t1);
  fp2_sub(u0, u0, t2);
  fp2_mul_xi(u0, u0);
  fp2_add(u0, u0, t0);
  fp2_add_lazy(s0, a(0), a(1));
  fp2_add_lazy(s1, b(0), b(1));
  fp2_mul(u1, s0, s1);
  fp2_sub(u1, u1, t0);
  fp2_sub(u1, u1, t1);
  fp2 x2;
  fp2_mul_xi(x2, t2);
  fp2_add(u1, u1, x2);
  fp2_add_lazy(s0, a(0), a(2));
  fp2_add_lazy(s1, b(0), b(2));
  fp2_mul(u2, s0, s1);
  fp2_sub(u2, u2, t0);
  fp2_sub(u2, u2, t2);
  fp2_add(u2, u2, t1);
  r.c0 = u0;
  r.c1 = u1;
  r.c2 = u2;
}
#endif

// f <- f^2 in place (fp12_sqr_inl's complex squaring).  t = a0 a1 first; then a0 + a1 and a0 + v a1 overwrite a0 and
// a1 (a1 held in registers for the pass), and their product s gives c0 = s - t - v t, c1 = 2t.
template <int S>
BLS_HD BLS_INLINE void fp12_sqr_l(const f12l<S>& F) {
  fp6 t;
  fp6_mul_fetch(t, [&](int i) { return F.ld(i); }, [&](int i) { return F.ld(3 + i); });
  {
    const fp2 b0 = F.ld(3), b1 = F.ld(4), b2 = F.ld(5);
    fp2 vb0, s, u;
    fp2_mul_xi(vb0, b2);  // v a1 = (xi a1.c2, a1.c0, a1.c1)
    fp2 a = F.ld(0);
    fp2_add(s, a, b0);
    fp2_add(u, a, vb0);
    F.st(0, s);
    F.st(3, u);
    a = F.ld(1);
    fp2_add(s, a, b1);
    fp2_add(u, a, b0);
    F.st(1, s);
    F.st(4, u);
    a = F.ld(2);
    fp2_add(s, a, b2);
    fp2_add(u, a, b1);
    F.st(2, s);
    F.st(5, u);
  }
  fp6 s;
  fp6_mul_fetch(s, [&](int i) { return F.ld(i); }, [&](int i) { return F.ld(3 + i); });
  fp6 vt;
  fp6_mul_v(vt, t);
  fp2 c;
  fp2_sub(c, s.c0, t.c0);
  fp2_sub(c, c, vt.c0);
  F.st(0, c);
  fp2_sub(c, s.c1, t.c1);
  fp2_sub(c, c, vt.c1);
  F.st(1, c);
  fp2_sub(c, s.c2, t.c2);
  fp2_sub(c, c, vt.c2);
  F.st(2, c);
  fp2_add(c, t.c0, t.c0);
  F.st(3, c);
  fp2_add(c, t.c1, t.c1);
  F.st(4, c);
  fp2_add(c, t.c2, t.c2);
  F.st(5, c);
}

// f <- f la lb in place (fp12_mul_line2_inl).  t0 = F0 L0 and t1 = F1 (x v + y v^2) read f; then F0 + F1 overwrites F1,
// the final c0 = t0 + v t1 overwrites F0, and c1 = (F0 + F1) l - (t0 + t1) overwrites F1.
template <int S>
BLS_HD BLS_INLINE void fp12_mul_line2_l(const f12l<S>& F, const fp2& ga0_in, const fp2& ga1_in, const fp2& ha1_in,
                                        const fp2& gb0_in, const fp2& gb1_in, const fp2& hb1_in) {
  const fp2 ga0 = ga0_in;
  const fp2 ga1 = ga1_in;
  const fp2 ha1 = ha1_in;
  const fp2 gb0 = gb0_in;
  const fp2 gb1 = gb1_in;
  const fp2 hb1 = hb1_in;
  fp2 p00, p11, phh, sa, sb, t;
  fp6 L0;
  fp2 x, y;
  fp2_mul(p00, ga0, gb0);
  fp2_mul(p11, ga1, gb1);
  fp2_mul(phh, ha1, hb1);
  fp2_add_lazy(sa, ga0, ga1);
  fp2_add_lazy(sb, gb0, gb1);
  fp2_mul(t, sa, sb);
  fp2_sub(t, t, p00);
  fp2_sub(L0.c1, t, p11);  // ga0 gb1 + ga1 gb0
  fp2_mul_xi(t, phh);
  fp2_add(L0.c0, p00, t);  // ga0 gb0 + xi ha1 hb1
  L0.c2 = p11;             // ga1 gb1
  fp2_add_lazy(sa, ga0, ha1);
  fp2_add_lazy(sb, gb0, hb1);
  fp2_mul(x, sa, sb);
  fp2_sub(x, x, p00);
  fp2_sub(x, x, phh);  // ga0 hb1 + ha1 gb0
  fp2_add_lazy(sa, ga1, ha1);
  fp2_add_lazy(sb, gb1, hb1);
  fp2_mul(y, sa, sb);
  fp2_sub(y, y, p11);
  fp2_sub(y, y, phh);  // ga1 hb1 + ha1 gb1
  fp6 t0, t1;
  fp6_mul_fetch(t0, [&](int i) { return F.ld(i); }, [&](int i) { return i == 0 ? L0.c0 : (i == 1 ? L0.c1 : L0.c2); });
#if BLS_LAZY_FP6
  {  // t1 = F1 (x v + y v^2) = xi(a1 y + a2 x) + (a0 x + xi a2 y) v + (a0 y + a1 x) v^2, one reduction per coefficient
    fp2 u, xa2;
    fp2_mul2(u, F.ld(4), y, F.ld(5), x);
    fp2_mul_xi(t1.c0, u);
    fp2_mul_xi(xa2, F.ld(5));
    fp2_mul2(t1.c1, F.ld(3), x, xa2, y);
    fp2_mul2(t1.c2, F.ld(3), y, F.ld(4), x);
  }
#else
  {  // t1 = F1 (x v + y v^2) = xi(a1 y + a2 x) + (a0 x + xi a2 y) v + (a0 y + a1 x) v^2
    fp2 m1, m2, m0, u, w2;
    fp2_mul(m1, F.ld(4), x);
    fp2_mul(m2, F.ld(5), y);
    fp2_mul(m0, F.ld(3), x);
    fp2_add_lazy(u, F.ld(4), F.ld(5));
    fp2_add_lazy(w2, x, y);
    fp2_mul(u, u, w2);
    fp2_sub(u, u, m1);
    fp2_sub(u, u, m2);
    fp2_mul_xi(t1.c0, u);
    fp2_mul_xi(u, m2);
    fp2_add(t1.c1, m0, u);
    fp2_mul(u, F.ld(3), y);
    fp2_add(t1.c2, u, m1);
  }
#endif
  fp2 c;
  for (int i = 0; i < 3; ++i) {  // F1 <- F0 + F1
    fp2_add(c, F.ld(i), F.ld(3 + i));
    F.st(3 + i, c);
  }
  fp6 d;
  {
    fp6 vt1;
    fp6_mul_v(vt1, t1);
    fp2_add(c, t0.c0, vt1.c0);
    F.st(0, c);
    fp2_add(c, t0.c1, vt1.c1);
    F.st(1, c);
    fp2_add(c, t0.c2, vt1.c2);
    F.st(2, c);
    fp6_add(d, t0, t1);
  }
  fp6 l, s;
  l.c0 = L0.c0;
  fp2_add(l.c1, L0.c1, x);
  fp2_add(l.c2, L0.c2, y);
  fp6_mul_fetch(s, [&](int i) { return F.ld(3 + i); }, [&](int i) { return i == 0 ? l.c0 : (i == 1 ? l.c1 : l.c2); });
  fp2_sub(c, s.c0, d.c0);
  F.st(3, c);
  fp2_sub(c, s.c1, d.c1);
  F.st(4, c);
  fp2_sub(c, s.c2, d.c2);
  F.st(5, c);
}

// fp6_mul_01 / fp6_mul_1 (tower.h) with a's coefficients fetched at each use.
template <class A>
BLS_HD BLS_INLINE void fp6_mul_01_fetch(fp6& r, const A& a, const fp2& b0, const fp2& b1) {
#if BLS_LAZY_FP6  // one reduction per coefficient: c0 = a0 b0 + (xi a2) b1, c1 = a0 b1 + a1 b0, c2 = a2 b0 + a1 b1
  fp2 xa2, c0, c1, c2;
  fp2_mul_xi(xa2, a(2));
  fp2_mul2(c0, a(0), b0, xa2, b1);
  fp2_mul2(c1, a(0), b1, a(1), b0);
  fp2_mul2(c2, a(2), b0, a(1), b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
#else
  fp2 t0, t1, s0, s1, u, c0, c1, c2;
  fp2_mul(t0, a(0), b0);
  fp2_mul(t1, a(1), b1);
  fp2_mul(u, a(2), b1);
  fp2_mul_xi(u, u);
  fp2_add(c0, u, t0);  // t0 + xi a2 b1
  fp2_add_lazy(s0, a(0), a(1));
  fp2_add(s1, b0, b1);
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);  // (a0 + a1)(b0 + b1) - t0 - t1
  fp2_mul(c2, a(2), b0);
  fp2_add(c2, c2, t1);  // a2 b0 + t1
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
#endif
}
template <class A>
BLS_HD BLS_INLINE void fp6_mul_1_fetch(fp6& r, const A& a, const fp2& b1) {
  fp2 c0;
  fp2_mul(c0, a(2), b1);
  fp2_mul_xi(r.c0, c0);
  fp2_mul(r.c1, a(0), b1);
  fp2_mul(r.c2, a(1), b1);
}

// f <- f l in place for one line (tower.h fp12_mul_line): t0 = F0 (g0 + g1 v), t1 = F1 (h1 v); F0 + F1 overwrites F1,
// c0 = t0 + v t1 overwrites F0, c1 = (F0 + F1)(g0 + (g1 + h1) v) - (t0 + t1) overwrites F1.
template <int S>
BLS_HD BLS_INLINE void fp12_mul_line_l(const f12l<S>& F, const fp2& g0_in, const fp2& g1_in, const fp2& h1_in) {
  const fp2 g0 = g0_in;
  const fp2 g1 = g1_in;
  const fp2 h1 = h1_in;
  fp6 t0, t1;
  fp6_mul_01_fetch(t0, [&](int i) { return F.ld(i); }, g0, g1);
  fp6_mul_1_fetch(t1, [&](int i) { return F.ld(3 + i); }, h1);
  fp2 c;
  for (int i = 0; i < 3; ++i) {  // F1 <- F0 + F1
    fp2_add(c, F.ld(i), F.ld(3 + i));
    F.st(3 + i, c);
  }
  fp6 d;
  {
    fp6 vt1;
    fp6_mul_v(vt1, t1);
    fp2_add(c, t0.c0, vt1.c0);
    F.st(0, c);
    fp2_add(c, t0.c1, vt1.c1);
    F.st(1, c);
    fp2_add(c, t0.c2, vt1.c2);
    F.st(2, c);
    fp6_add(d, t0, t1);
  }
  fp2 gh1;
  fp2_add(gh1, g1, h1);
  fp6 s;
  fp6_mul_01_fetch(s, [&](int i) { return F.ld(3 + i); }, g0, gh1);
  fp2_sub(c, s.c0, d.c0);
  F.st(3, c);
  fp2_sub(c, s.c1, d.c1);
  F.st(4, c);
  fp2_sub(c, s.c2, d.c2);
  F.st(5, c);
}

// miller_loop_2 (pairing.h) with f in LDS; f_out and T1_out as there.
// Register-allocation hint: x's dwords pass through an empty asm statement in accumulation registers, so the
// allocator keeps a value that waits across a doubling step in AGPRs rather than in scratch.
// Round 6: 6 (T0 and the first pair's line coefficients parked after its doubling step, P0 at the loop top). With
// the loop inlined into k_verify_fused (op_verify_l_kernel) the parked values stay in AGPRs instead of scratch:
// same-box A/B C2 1.854M -> 1.865M/s (profiles/r06/c2_park_ab.json; 2 alone +0.6 %, 4 alone +0.4 %).
#ifndef BLS_ML_PARK
#define BLS_ML_PARK 6
#endif
template <class T>
BLS_HD BLS_INLINE void park_agpr(T& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t* w = reinterpret_cast<uint32_t*>(&x);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) asm("" : "+a"(w[i]));
#endif
}

#ifndef BLS_ML_DBL
#define BLS_ML_DBL miller_dbl_step_inl
#endif
#ifndef BLS_MILLER_L_CALL
#define BLS_MILLER_L_CALL BLS_CALL
#endif
// P1_NEG_GEN: P1 is -g1 (Verify's second pair), so its coordinates are immediates rematerialized at each use instead
// of 24 registers live across the loop.
// The loop's body is an inline function: miller_loop_2_l below is its out-of-line form (the RLC and keyed kernels call
// it), and k_verify_fused inlines the body into the kernel itself (ops.h op_verify_l_kernel), where no callee-saved
// register set applies: the loop then spills to all 256 AGPRs before scratch (225 scratch instructions per doubling
// iteration instead of 275, C2 +0.5 %).
template <int S, bool P1_NEG_GEN = false>
BLS_HD BLS_INLINE void miller_loop_2_l_body(fp12& f_out, const f12l<S> F, const g1a& P0_in, const g2a& Q0,
                                          const g1a& P1_in, const g2a& Q1, g2j* T1_out) {
  g1a P0 = P0_in;
  g1a P1;
  if (P1_NEG_GEN) {
    P1.x = G1_GEN_X;
    P1.y = G1_NEG_GEN_Y;
  } else {
    P1 = P1_in;
  }
  g2j T0, T1;
  T0.x = Q0.x;
  T0.y = Q0.y;
  fp2_set_one(T0.z);
  T1.x = Q1.x;
  T1.y = Q1.y;
  fp2_set_one(T1.z);
  {
    fp12 f;
    fp2 a0, a1, ah, g0, g1, h1;
    miller_dbl_step_inl(T0, a0, a1, ah, P0.x, P0.y);
    miller_dbl_step_inl(T1, g0, g1, h1, P1.x, P1.y);
    fp12_line_pair(f, a0, a1, ah, g0, g1, h1);
    F.st12(f);
    miller_add_step_inl(T0, a0, a1, ah, Q0, P0.x, P0.y);  // bit 62 of |x| is set
    miller_add_step_inl(T1, g0, g1, h1, Q1, P1.x, P1.y);
    fp12_mul_line2_l(F, a0, a1, ah, g0, g1, h1);
  }
  for (int bit = 61; bit >= 0; --bit) {
#if BLS_ML_PARK & 1
    park_agpr(T0);
    park_agpr(T1);
#endif
#if BLS_ML_PARK & 4
    park_agpr(P0);
#endif
    fp12_sqr_l(F);
    fp2 a0, a1, ah, g0, g1, h1;
    BLS_ML_DBL(T0, a0, a1, ah, P0.x, P0.y);
#if BLS_ML_PARK & 2
    park_agpr(T0);
    park_agpr(a0);
    park_agpr(a1);
    park_agpr(ah);
#endif
    BLS_ML_DBL(T1, g0, g1, h1, P1.x, P1.y);
    fp12_mul_line2_l(F, a0, a1, ah, g0, g1, h1);
    if ((X_ABS >> bit) & 1ull) {
      miller_add_step_inl(T0, a0, a1, ah, Q0, P0.x, P0.y);
      miller_add_step_inl(T1, g0, g1, h1, Q1, P1.x, P1.y);
      fp12_mul_line2_l(F, a0, a1, ah, g0, g1, h1);
    }
  }
  fp12 f;
  F.ld12(f);
  fp12_conj(f_out, f);
  if (T1_out) *T1_out = T1;
}
template <int S, bool P1_NEG_GEN = false>
BLS_HD BLS_MILLER_L_CALL void miller_loop_2_l(fp12& f_out, const f12l<S> F, const g1a& P0_in, const g2a& Q0, const g1a& P1_in,
                                     const g2a& Q1, g2j* T1_out) {
  miller_loop_2_l_body<S, P1_NEG_GEN>(f_out, F, P0_in, Q0, P1_in, Q1, T1_out);
}

// f <- f b in place, b dense in registers (fp12_mul_inl): t0 = F0 b0, t1 = F1 b1; F0 + F1 overwrites F1, c0 = t0 + v t1
// overwrites F0, c1 = (F0 + F1)(b0 + b1) - (t0 + t1) overwrites F1.
template <int S>
BLS_HD BLS_INLINE void fp12_mul_l(const f12l<S>& F, const fp12& b) {
  fp6 t0, t1;
  fp6_mul_fetch(t0, [&](int i) { return F.ld(i); }, [&](int i) { return i == 0 ? b.c0.c0 : (i == 1 ? b.c0.c1 : b.c0.c2); });
  fp6_mul_fetch(t1, [&](int i) { return F.ld(3 + i); }, [&](int i) { return i == 0 ? b.c1.c0 : (i == 1 ? b.c1.c1 : b.c1.c2); });
  fp2 c;
  for (int i = 0; i < 3; ++i) {  // F1 <- F0 + F1
    fp2_add(c, F.ld(i), F.ld(3 + i));
    F.st(3 + i, c);
  }
  fp6 d, sb;
  {
    fp6 vt1;
    fp6_mul_v(vt1, t1);
    fp2_add(c, t0.c0, vt1.c0);
    F.st(0, c);
    fp2_add(c, t0.c1, vt1.c1);
    F.st(1, c);
    fp2_add(c, t0.c2, vt1.c2);
    F.st(2, c);
    fp6_add(d, t0, t1);
  }
  fp6_add(sb, b.c0, b.c1);
  fp6 s;
  fp6_mul_fetch(s, [&](int i) { return F.ld(3 + i); }, [&](int i) { return i == 0 ? sb.c0 : (i == 1 ? sb.c1 : sb.c2); });
  fp2_sub(c, s.c0, d.c0);
  F.st(3, c);
  fp2_sub(c, s.c1, d.c1);
  F.st(4, c);
  fp2_sub(c, s.c2, d.c2);
  F.st(5, c);
}

// fp12_cyc_exp_xabs_karabina (pairing.h) with the decompressed powers' product accumulated in LDS: the tail's
// accumulator (144 dwords) no longer shares the registers with the power being decompressed and the saved states.
// Returns true, leaving r untouched, in the degenerate case: the caller then takes the Granger-Scott exponentiation
// (fp12_cyc_exp_xabs_l), so that rarely used call chain adds to the caller's stack depth, not to this one's -- every
// kernel's private segment is sized by its deepest chain (~3 KB less per lane here).
template <int S>
BLS_HD BLS_CALL bool fp12_cyc_exp_xabs_karabina_l(fp12& r, const fp12& a_in, const f12l<S> F) {
  static_assert(X_ABS == 0xd201000000010000ull, "the squaring counts below are |x|'s set bits");
  cyc_c st[6];  // a^(2^k) for k = 16, 48, 57, 60, 62, 63
  cyc_c c;
  c.z2 = a_in.c1.c0;
  c.z3 = a_in.c0.c2;
  c.z4 = a_in.c0.c1;
  c.z5 = a_in.c1.c2;
  cyc_sqr_run(c, 16);
  st[0] = c;
  cyc_sqr_run(c, 32);
  st[1] = c;
  cyc_sqr_run(c, 9);
  st[2] = c;
  cyc_sqr_run(c, 3);
  st[3] = c;
  cyc_sqr_run(c, 2);
  st[4] = c;
  cyc_sqr_run(c, 1);
  st[5] = c;
  fp2 num[6], den[6], pre[6];
  int s;
#pragma unroll 1
  for (s = 0; s < 6; ++s) cyc_z1_parts(num[s], den[s], st[s]);
  pre[0] = den[0];
#pragma unroll 1
  for (s = 1; s < 6; ++s) fp2_mul(pre[s], pre[s - 1], den[s]);
  if (fp2_is_zero(pre[5])) return true;  // practically never: the identity or z2 = z3 = 0 at one of the six powers
  fp2 inv;
  fp2_inv(inv, pre[5]);
#pragma unroll 1
  for (s = 5; s >= 0; --s) {
    fp2 is, z1;
    if (s > 0) {
      fp2_mul(is, inv, pre[s - 1]);  // 1 / den[s]
      fp2_mul(inv, inv, den[s]);
    } else {
      is = inv;
    }
    fp2_mul(z1, num[s], is);
    fp12 d;
    cyc_decompress(d, st[s], z1);
    if (s == 5)
      F.st12(d);
    else
      fp12_mul_l(F, d);
  }
  F.ld12(r);
  return false;
}
template <int S>
BLS_HD BLS_INLINE void fp12_cyc_exp_xabs_l(fp12& r, const fp12& a_in, const f12l<S>& F) {
  if (fp12_cyc_exp_xabs_karabina_l(r, a_in, F)) fp12_cyc_exp_xabs_gs(r, a_in);
}

// final_exponentiation (pairing.h) with the a^|x| powers on fp12_cyc_exp_xabs_karabina_l; F is free scratch here.
template <int S>
BLS_HD BLS_CALL void final_exponentiation_l(fp12& r, const fp12& f_in, const f12l<S> F) {
  // The temporaries are scoped so their stack slots can share space: every Fp12 here is passed by address to a real
  // call, so it lives in the frame, and at function scope each one held its own 576 B for the whole function (the
  // frame is part of every verify kernel's private segment).  f_in is read only by the easy part and r written only
  // at the end, so r may alias f_in.
  fp12 m;
  {  // easy part: f^((p^6-1)(p^2+1))
    fp12 t, fi;
    fp12_conj(t, f_in);
    fp12_inv(fi, f_in);
    BLS_FE_MUL(m, t, fi);
    fp12_frobenius(t, m, 2);
    BLS_FE_MUL(m, t, m);
  }
  fp12 t1;
  {  // t0 = m^((x-1)^2), t1 = t0^(x+p)
    fp12 t0, u;
    fp12_cyc_exp_xabs_l(t0, m, F);
    BLS_FE_MUL(t0, t0, m);
    fp12_conj(t0, t0);
    fp12_cyc_exp_xabs_l(u, t0, F);
    BLS_FE_MUL(u, u, t0);
    fp12_conj(t0, u);
    fp12_cyc_exp_xabs_l(u, t0, F);
    fp12_conj(u, u);
    fp12_frobenius(t1, t0, 1);
    BLS_FE_MUL(t1, t1, u);
  }
  fp12 t2;
  {  // t2 = t1^(x^2+p^2-1)
    fp12 u;
    fp12_cyc_exp_xabs_l(u, t1, F);
    fp12_cyc_exp_xabs_l(u, u, F);
    fp12_frobenius(t2, t1, 2);
    BLS_FE_MUL(t2, t2, u);
    fp12_conj(u, t1);
    BLS_FE_MUL(t2, t2, u);
  }
  {  // r = t2 m^3
    fp12 u;
    fp12_cyclotomic_sqr(u, m);
    BLS_FE_MUL(u, u, m);
    BLS_FE_MUL(r, t2, u);
  }
}
#ifndef BLS_FE_LDS
#define BLS_FE_LDS 1
#endif
template <int S>
BLS_HD BLS_INLINE void final_exp_l(fp12& r, const fp12& f, const f12l<S>& F) {
#if BLS_FE_LDS
  final_exponentiation_l(r, f, F);
#else
  final_exponentiation(r, f);
#endif
}

// e(pk, hm) e(-g1, sig) == 1 on decoded points (ops.h pairing_check_verify) with f in LDS.
template <int S>
BLS_HD BLS_CALL bool pairing_check_verify_l(const g1a& pk, const g2a& hm, const g2a& sig, const f12l<S> F) {
  g1a P1;
  P1.x = G1_GEN_X;
  P1.y = G1_NEG_GEN_Y;
  fp12 f;
  miller_loop_2_l<S, true>(f, F, pk, hm, P1, sig, nullptr);
  final_exp_l(f, f, F);  // in place (final_exponentiation_l allows r == f_in)
  return fp12_is_one(f);
}

}  // namespace bls
