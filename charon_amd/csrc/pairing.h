// Optimal ate pairing on BLS12-381: multi-Miller loop with homogeneous projective steps on the
// M-type twist and sparse line multiplication, then the shared final exponentiation
// (easy part + Hayashida-Hayasaka-Teruya hard part, which yields e(P,Q)^3 -- harmless for a
// "== 1" product check because gcd(3, r) = 1).
//
// Replaces the pairing check inside herumi's blsVerify (tbls/herumi.go:298 VerifyByte) and
// FastAggregateVerify (herumi.go:334).
#pragma once
#include "curve.h"

namespace bls {

struct g1_pair_in {  // P in affine coordinates, or is_inf
  fp x, y;
  bool is_inf;
};

// Doubling step T <- 2T; returns the tangent line at T evaluated at P, in the sparse form
// (g0 + g1 v) + (h1 v) w  with  g0 = 3b'Z^2 - Y^2, g1 = 3X^2 x_P, h1 = -2YZ y_P.
// Addition step T <- T + Q (Q affine); line (theta x2 - lambda y2) + (-theta x_P) v + (lambda y_P) v w

// f = prod_i f_{|x|, Q_i}(P_i), conjugated (x < 0).  Pairs with an infinity input contribute 1.

// r = f^((p^12-1)/r * 3)

// The products are asm statements the compiler does not reorder, so the source order is the schedule: each temporary
// dies soon after it is made (peak: five Fp2 temporaries and the line coefficients; computing A..J first kept eight
// live, and the Miller loop spilled them: 16 % fewer scratch instructions in the loop body).
BLS_HD BLS_INLINE void miller_dbl_step_inl(g2j& T_in, fp2& g0, fp2& g1, fp2& h1, const fp& xp_in, const fp& yp_in) {
  const fp xp = xp_in;
  const fp yp = yp_in;
  g2j T = T_in;
  // Homogeneous coordinates (x = X/Z, y = Y/Z).  Note: T.z here is the projective Z, not Jacobian.
  fp2 A, B, C, E, H, t;
  fp2_sqr(t, T.x);  // J = X^2
  {
    fp2 J3;
    fp2_add(J3, t, t);
    fp2_add(J3, J3, t);
    fp2_mul_fp(g1, J3, xp);  // g1 = 3 X^2 x_P
  }
  fp2_mul(A, T.x, T.y);
  fp2_half(A, A);  // A = XY/2
  fp2_sqr(C, T.z);
  fp2_mul_3b2(E, C);  // E = 3b' Z^2 (additions, not a product)
  fp2_add(H, T.y, T.z);
  fp2_sqr(H, H);
  fp2_sqr(B, T.y);
  fp2_sub(H, H, B);
  fp2_sub(H, H, C);  // H = 2YZ
  fp2_sub(g0, E, B);  // g0 = 3b' Z^2 - Y^2
  fp2_mul_fp(h1, H, yp);
  fp2_neg(h1, h1);  // h1 = -2YZ y_P
  fp2_mul(T.z, B, H);  // Z3 = B H
  fp2 F;
  fp2_add(F, E, E);
  fp2_add(F, F, E);  // F = 3E
  fp2_sub(t, B, F);
  fp2_mul(T.x, A, t);  // X3 = A (B - F)
  fp2_add(t, B, F);
  fp2_half(t, t);  // G = (B + F)/2
  fp2_sqr(t, t);
  fp2 E2;
  fp2_sqr(E2, E);
  fp2_add(C, E2, E2);
  fp2_add(C, C, E2);
  fp2_sub(T.y, t, C);  // Y3 = G^2 - 3 E^2
  T_in = T;
}
BLS_HD BLS_MILLER_CALL void miller_dbl_step(g2j& T_in, fp2& g0, fp2& g1, fp2& h1, const fp& xp_in, const fp& yp_in) { miller_dbl_step_inl(T_in, g0, g1, h1, xp_in, yp_in); }

// Low-liveness order as in the doubling step: the line coefficients first, then each temporary consumed right away.
BLS_HD BLS_INLINE void miller_add_step_inl(g2j& T_in, fp2& g0, fp2& g1, fp2& h1, const g2a& Q_in, const fp& xp_in,
                                         const fp& yp_in) {
  const fp xp = xp_in;
  const fp yp = yp_in;
  g2j T = T_in;
  fp2 theta, lambda, t, u;
  fp2_mul(t, Q_in.y, T.z);
  fp2_sub(theta, T.y, t);  // theta = Y - y2 Z
  fp2_mul(t, Q_in.x, T.z);
  fp2_sub(lambda, T.x, t);  // lambda = X - x2 Z
  // line
  fp2_mul(t, theta, Q_in.x);
  fp2_mul(u, lambda, Q_in.y);
  fp2_sub(g0, t, u);
  fp2_mul_fp(g1, theta, xp);
  fp2_neg(g1, g1);
  fp2_mul_fp(h1, lambda, yp);
  // point
  fp2 C, D, E, G;
  fp2_sqr(C, theta);
  fp2_mul(C, T.z, C);  // F = Z theta^2
  fp2_sqr(D, lambda);
  fp2_mul(G, T.x, D);  // G = X lambda^2
  fp2_mul(E, lambda, D);  // E = lambda^3
  fp2_mul(T.z, T.z, E);  // Z3 = Z E
  fp2_mul(t, T.y, E);  // Y E
  fp2_add(u, E, C);
  fp2_sub(u, u, G);
  fp2_sub(u, u, G);  // H = E + F - 2G
  fp2_mul(T.x, lambda, u);  // X3 = lambda H
  fp2_sub(u, G, u);
  fp2_mul(u, theta, u);
  fp2_sub(T.y, u, t);  // Y3 = theta (G - H) - Y E
  T_in = T;
}
BLS_HD BLS_MILLER_CALL void miller_add_step(g2j& T_in, fp2& g0, fp2& g1, fp2& h1, const g2a& Q_in, const fp& xp_in,
                                         const fp& yp_in) { miller_add_step_inl(T_in, g0, g1, h1, Q_in, xp_in, yp_in); }

// Fused 2-pair Miller iterations: one call per step instead of four, so f, T0, T1 cross the stack once per step
// and one prologue saves the callee-saved registers instead of four (each Fp12-level function saves ~180 of
// them).  BLS_MILLER_FUSE = 1: squaring + both doubling steps + line-pair product in one call; 2: the squaring
// stays a separate call.
#ifndef BLS_MILLER_FUSE
#define BLS_MILLER_FUSE 0
#endif
BLS_HD BLS_CALL void miller_dbl2_line2(fp12& f_io, g2j& T0_io, g2j& T1_io, const g1a& P0_in, const g1a& P1_in,
                                       bool square) {
  fp12 f = f_io;
  g2j T0 = T0_io, T1 = T1_io;
  const g1a P0 = P0_in, P1 = P1_in;
  if (square) {
    fp12 s;
    fp12_sqr_inl(s, f);
    f = s;
  }
  fp2 a0, a1, ah, g0, g1, h1;
  miller_dbl_step_inl(T0, a0, a1, ah, P0.x, P0.y);
  miller_dbl_step_inl(T1, g0, g1, h1, P1.x, P1.y);
  fp12_mul_line2_inl(f, a0, a1, ah, g0, g1, h1);
  f_io = f;
  T0_io = T0;
  T1_io = T1;
}

// The 2-pair loop of Verify (both pairs live) on its own: one code path for the register allocator, T0/T1/f/P in the
// loop's registers, and the first step's f = 1 * la * lb formed from the line product alone (6 Fp2 products, not 23).
// T1_out (when given) receives the second pair's final T = [|x|] Q1 in homogeneous coordinates, with Z = 0 if any
// step was exceptional (see g2_subgroup_from_miller).
BLS_HD BLS_CALL void miller_loop_2(fp12& f_out, const g1a& P0_in, const g2a& Q0, const g1a& P1_in, const g2a& Q1,
                                   g2j* T1_out = nullptr) {
  const g1a P0 = P0_in, P1 = P1_in;
  g2j T0, T1;
  T0.x = Q0.x;
  T0.y = Q0.y;
  fp2_set_one(T0.z);
  T1.x = Q1.x;
  T1.y = Q1.y;
  fp2_set_one(T1.z);
  fp12 f;
  {
    fp2 a0, a1, ah, g0, g1, h1;
    miller_dbl_step_inl(T0, a0, a1, ah, P0.x, P0.y);
    miller_dbl_step_inl(T1, g0, g1, h1, P1.x, P1.y);
    fp12_line_pair(f, a0, a1, ah, g0, g1, h1);
    miller_add_step_inl(T0, a0, a1, ah, Q0, P0.x, P0.y);  // bit 62 of |x| is set
    miller_add_step_inl(T1, g0, g1, h1, Q1, P1.x, P1.y);
    fp12_mul_line2_inl(f, a0, a1, ah, g0, g1, h1);
  }
  for (int bit = 61; bit >= 0; --bit) {
    fp12_sqr_inl(f, f);
    fp2 a0, a1, ah, g0, g1, h1;
    miller_dbl_step_inl(T0, a0, a1, ah, P0.x, P0.y);
    miller_dbl_step_inl(T1, g0, g1, h1, P1.x, P1.y);
    fp12_mul_line2_inl(f, a0, a1, ah, g0, g1, h1);
    if ((X_ABS >> bit) & 1ull) {
      miller_add_step_inl(T0, a0, a1, ah, Q0, P0.x, P0.y);
      miller_add_step_inl(T1, g0, g1, h1, Q1, P1.x, P1.y);
      fp12_mul_line2_inl(f, a0, a1, ah, g0, g1, h1);
    }
  }
  fp12_conj(f_out, f);
  if (T1_out) *T1_out = T1;
}

// The signature's G2 membership from the Miller loop's by-product (Scott 2021: Q in G2 iff psi(Q) = [x] Q).  The loop
// runs T over |x|'s bits from T = Q, so without an exceptional step T ends as [|x|] Q = -[x] Q.  The homogeneous
// steps are exceptional exactly when their Z comes out 0 (doubling: Y = 0 or Z = 0; addition: T = +-Q, lambda = 0),
// and Z stays 0 afterwards; an exceptional step means [k]Q in {O, +-Q} for some k < 2^64, i.e. Q of small order, not in
// G2.  So Q (affine, not infinity) is in G2 iff Z != 0 and T = -psi(Q): X = psi_x Z, Y = -psi_y Z.  This replaces the
// 63-doubling scalar multiplication of g2_in_subgroup for Verify's signature.
BLS_HD BLS_INLINE bool g2_subgroup_from_miller(const g2j& T, const g2a& Q) {
  g2j q, ps;
  jac_from_aff(q, Q);
  g2_psi(ps, q);  // affine in, z = 1 out
  fp2 t;
  bool ok = !fp2_is_zero(T.z);
  fp2_mul(t, ps.x, T.z);
  ok = ok && fp2_eq(t, T.x);
  fp2_mul(t, ps.y, T.z);
  fp2_add(t, t, T.y);
  return ok && fp2_is_zero(t);
}

BLS_HD BLS_CALL void miller_loop_n(fp12& f, const g1a* P, const g2a* Q, const bool* skip, int n) {
  static_assert((X_ABS >> 62) & 1ull, "miller_loop_2 folds the top bit below |x|'s leading one into its first step");
  if (n == 2 && !skip[0] && !skip[1]) {
    miller_loop_2(f, P[0], Q[0], P[1], Q[1]);
    return;
  }
  constexpr int MAXN = 2;
  g2j T[MAXN];
  for (int i = 0; i < n; ++i) {
    T[i].x = Q[i].x;
    T[i].y = Q[i].y;
    fp2_set_one(T[i].z);
  }
  fp12_set_one(f);
  fp2 g0, g1, h1;
  bool first = true;
  for (int bit = 62; bit >= 0; --bit) {
    if (n == 2 && !skip[0] && !skip[1]) {  // both lines live: one line-pair product (fp12_mul_line2)
      fp2 a0, a1, ah;
#if BLS_MILLER_FUSE == 1
      miller_dbl2_line2(f, T[0], T[1], P[0], P[1], !first);
#elif BLS_MILLER_FUSE == 2
      if (!first) fp12_sqr(f, f);
      miller_dbl2_line2(f, T[0], T[1], P[0], P[1], false);
#else
      if (!first) fp12_sqr(f, f);
      miller_dbl_step(T[0], a0, a1, ah, P[0].x, P[0].y);
      miller_dbl_step(T[1], g0, g1, h1, P[1].x, P[1].y);
      fp12_mul_line2(f, a0, a1, ah, g0, g1, h1);
#endif
      first = false;
      if ((X_ABS >> bit) & 1ull) {
        miller_add_step(T[0], a0, a1, ah, Q[0], P[0].x, P[0].y);
        miller_add_step(T[1], g0, g1, h1, Q[1], P[1].x, P[1].y);
        fp12_mul_line2(f, a0, a1, ah, g0, g1, h1);
      }
      continue;
    }
    if (!first) fp12_sqr(f, f);
    first = false;
    for (int i = 0; i < n; ++i) {
      miller_dbl_step(T[i], g0, g1, h1, P[i].x, P[i].y);
      if (!skip[i]) fp12_mul_line(f, g0, g1, h1);
    }
    if ((X_ABS >> bit) & 1ull) {
      for (int i = 0; i < n; ++i) {
        miller_add_step(T[i], g0, g1, h1, Q[i], P[i].x, P[i].y);
        if (!skip[i]) fp12_mul_line(f, g0, g1, h1);
      }
    }
  }
  fp12_conj(f, f);
}

#ifndef BLS_EXP_MUL
#define BLS_EXP_MUL fp12_mul
#endif

// ---- Karabina's compressed cyclotomic squaring ("Squaring in cyclotomic subgroups", Math. Comp. 2013) ----------
// With Fp12 = Fp4[w]/(w^3 - s), Fp4 = Fp2[s]/(s^2 - xi), an element is (z0 + z1 s) + (z2 + z3 s) w + (z4 + z5 s) w^2
// (z0 = c0.c0, z1 = c1.c1, z2 = c1.c0, z3 = c0.c2, z4 = c0.c1, z5 = c1.c2: the Granger-Scott pairs of
// fp12_cyclotomic_sqr_body).  Granger-Scott's new (z2..z5) depend on (z2..z5) alone, so a run of squarings can carry
// only those four: 6 Fp2 squarings per squaring instead of 9.  (z0, z1) come back from the cyclotomic relations:
//   z2 != 0:  z1 = (xi z5^2 + 3 z4^2 - 2 z3) / (4 z2)          z2 == 0:  z1 = 2 z4 z5 / z3
//   z0 = (2 z1^2 + z2 z5 - 3 z3 z4) xi + 1
// a^|x| is the product of a^(2^k) over |x|'s six set bits k = 16, 48, 57, 60, 62, 63, decompressed together with one
// Fp2 inversion (Montgomery's batch trick).  A lane whose denominators vanish (z2 = z3 = 0: the identity and a
// negligible set of other elements) takes the Granger-Scott exponentiation instead, so results are exact on all inputs.
struct cyc_c {
  fp2 z2, z3, z4, z5;
};
// The compressed state is small (96 dwords), so here the Fp2 squaring routine's pinned registers cost nothing
// (op_probe: fp12_cyc_exp_xabs 5.40M -> 5.31M cycles against 5.53M for Granger-Scott).
#ifndef BLS_KAR_FP2_SQR
#define BLS_KAR_FP2_SQR fp2_sqr
#endif
// The six decompressed powers are multiplied with the Fp12 product inlined: across a call its two 576-byte operands
// and result go through the stack (op_probe: fp12_cyc_exp_xabs 5.32M -> 4.75M cycles).
#ifndef BLS_KAR_MUL
#define BLS_KAR_MUL fp12_mul_inl
#endif
#ifndef BLS_FE_MUL
#define BLS_FE_MUL fp12_mul
#endif
BLS_HD BLS_INLINE void cyc_sqr_compressed(cyc_c& c) {
  fp2 s2, s3, s4, s5, t, u, v;
  BLS_KAR_FP2_SQR(s2, c.z2);
  BLS_KAR_FP2_SQR(s3, c.z3);
  BLS_KAR_FP2_SQR(s4, c.z4);
  BLS_KAR_FP2_SQR(s5, c.z5);
  fp2_add(t, c.z4, c.z5);
  BLS_KAR_FP2_SQR(t, t);
  fp2_sub(t, t, s4);
  fp2_sub(t, t, s5);  // 2 z4 z5
  fp2_add(u, c.z2, c.z3);
  BLS_KAR_FP2_SQR(u, u);
  fp2_sub(u, u, s2);
  fp2_sub(u, u, s3);  // 2 z2 z3
  // z2' = 2 z2 + 3 xi (2 z4 z5)
  fp2_mul_xi(t, t);
  fp2_add(v, c.z2, t);
  fp2_add(v, v, v);
  fp2_add(c.z2, v, t);
  // z3' = 3 (z4^2 + xi z5^2) - 2 z3
  fp2_mul_xi(s5, s5);
  fp2_add(s4, s4, s5);
  fp2_sub(v, s4, c.z3);
  fp2_add(v, v, v);
  fp2_add(c.z3, v, s4);
  // z4' = 3 (z2^2 + xi z3^2) - 2 z4
  fp2_mul_xi(s3, s3);
  fp2_add(s2, s2, s3);
  fp2_sub(v, s2, c.z4);
  fp2_add(v, v, v);
  fp2_add(c.z4, v, s2);
  // z5' = 2 z5 + 3 (2 z2 z3)
  fp2_add(v, c.z5, u);
  fp2_add(v, v, v);
  fp2_add(c.z5, v, u);
}
BLS_HD BLS_INLINE void fp2_select(fp2& r, uint32_t m, const fp2& a, const fp2& b) {  // m ? a : b (m a lane mask)
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    r.c0.v[i] = gcd30::bfi(m, a.c0.v[i], b.c0.v[i]);
    r.c1.v[i] = gcd30::bfi(m, a.c1.v[i], b.c1.v[i]);
  }
}
// z1 = num / den for one compressed element (den != 0 unless the lane is degenerate)
BLS_HD BLS_INLINE void cyc_z1_parts(fp2& num, fp2& den, const cyc_c& c) {
  const uint32_t nz = fp2_is_zero(c.z2) ? 0u : ~0u;
  fp2 a, b, t;
  BLS_CYC_FP2_SQR(a, c.z5);
  fp2_mul_xi(a, a);
  BLS_CYC_FP2_SQR(t, c.z4);
  fp2_add(a, a, t);
  fp2_add(a, a, t);
  fp2_add(a, a, t);
  fp2_sub(a, a, c.z3);
  fp2_sub(a, a, c.z3);  // xi z5^2 + 3 z4^2 - 2 z3
  fp2_mul(b, c.z4, c.z5);
  fp2_add(b, b, b);  // 2 z4 z5
  fp2_select(num, nz, a, b);
  fp2_add(t, c.z2, c.z2);
  fp2_add(t, t, t);  // 4 z2
  fp2_select(den, nz, t, c.z3);
}
BLS_HD BLS_INLINE void cyc_decompress(fp12& r, const cyc_c& c, const fp2& z1) {
  fp2 t, u, z0;
  BLS_CYC_FP2_SQR(t, z1);
  fp2_add(t, t, t);
  fp2_mul(u, c.z2, c.z5);
  fp2_add(t, t, u);
  fp2_mul(u, c.z3, c.z4);
  fp2_sub(t, t, u);
  fp2_sub(t, t, u);
  fp2_sub(t, t, u);
  fp2_mul_xi(t, t);
  fp2 one;
  fp2_set_one(one);
  fp2_add(z0, t, one);
  r.c0.c0 = z0;
  r.c1.c1 = z1;
  r.c1.c0 = c.z2;
  r.c0.c2 = c.z3;
  r.c0.c1 = c.z4;
  r.c1.c2 = c.z5;
}
BLS_HD BLS_CALL void fp12_cyc_exp_xabs_gs(fp12& r, const fp12& a_in);
#ifndef BLS_KAR_SQR_RUNS
#define BLS_KAR_SQR_RUNS 1
#endif
// n compressed squarings in place (a wave-uniform count)
BLS_HD BLS_CALL void cyc_sqr_run(cyc_c& c_io, int n) {
  cyc_c c = c_io;
#pragma unroll 1
  for (int k = 0; k < n; ++k) cyc_sqr_compressed(c);
  c_io = c;
}
// r = a^|x| for a in the cyclotomic subgroup, by compressed squarings
// Inlined into the final exponentiation's five call sites it measured slower (C2 1.710M -> 1.685M verifies/s; with
// the nine FE products inlined too 1.666M, profiles/r02_sched_variants.txt), so it stays a call.
#ifndef BLS_KAR_EXP_CALL
#define BLS_KAR_EXP_CALL BLS_CALL
#endif
BLS_HD BLS_KAR_EXP_CALL void fp12_cyc_exp_xabs_karabina(fp12& r, const fp12& a_in) {
  static_assert(X_ABS == 0xd201000000010000ull, "the squaring counts below are |x|'s set bits");
  cyc_c st[6];  // a^(2^k) for k = 16, 48, 57, 60, 62, 63
  cyc_c c;
  c.z2 = a_in.c1.c0;
  c.z3 = a_in.c0.c2;
  c.z4 = a_in.c0.c1;
  c.z5 = a_in.c1.c2;
#if BLS_KAR_SQR_RUNS
  // the squarings in runs between |x|'s set bits, each run a call of its own (cyc_sqr_run): inside it only the
  // compressed state is live, so the loop needs no scratch; inlined here, the allocator spilled around every
  // squaring for the sake of the decompression code below (33 scratch instructions per squaring)
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
  int s;
#else
  // one squaring loop with the save points as a wave-uniform test (one inlined copy of the squaring)
  int s = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; ++k) {
    cyc_sqr_compressed(c);
    if (k == 16 || k == 48 || k == 57 || k == 60 || k == 62 || k == 63) st[s++] = c;
  }
#endif
  // batch inversion of the six z1 denominators
  fp2 num[6], den[6], pre[6];
#pragma unroll 1
  for (s = 0; s < 6; ++s) cyc_z1_parts(num[s], den[s], st[s]);
  pre[0] = den[0];
#pragma unroll 1
  for (s = 1; s < 6; ++s) fp2_mul(pre[s], pre[s - 1], den[s]);
  const bool degenerate = fp2_is_zero(pre[5]);
  fp2 inv;
  fp2_inv(inv, pre[5]);
  fp12 acc, d;
#pragma unroll
  for (s = 5; s >= 0; --s) {
    fp2 is, z1;
    if (s > 0) {
      fp2_mul(is, inv, pre[s - 1]);  // 1 / den[s]
      fp2_mul(inv, inv, den[s]);
    } else {
      is = inv;
    }
    fp2_mul(z1, num[s], is);
    if (s == 5) {
      cyc_decompress(acc, st[s], z1);
    } else {
      cyc_decompress(d, st[s], z1);
      fp12 x = acc;
      BLS_KAR_MUL(acc, x, d);
    }
  }
  if (degenerate) {  // practically never: the identity or z2 = z3 = 0 at one of the six powers
    fp12_cyc_exp_xabs_gs(acc, a_in);
  }
  r = acc;
}
// r = a^|x| for a in the cyclotomic subgroup
// The base is NOT copied in: it is needed only by the 5 multiplications, so it stays in the caller's frame and
// fp12_mul reads it there, leaving the register file to the squaring chain (a register copy of it spilled
// inside the loop).  Likewise the accumulator's address is never taken, so it is not pinned to the stack.
BLS_HD BLS_CALL void fp12_cyc_exp_xabs_gs(fp12& r, const fp12& a_in) {
  fp12 acc = a_in;
  for (int bit = 62; bit >= 0; --bit) {
    fp12 t;
    fp12_cyclotomic_sqr_body(t, acc);  // inlined: acc stays in registers between squarings
    acc = t;
    if ((X_ABS >> bit) & 1ull) {  // through temporaries: taking acc's address would pin it to the stack
      fp12 x = acc, y;
      BLS_EXP_MUL(y, x, a_in);
      acc = y;
    }
  }
  r = acc;
}

#ifndef BLS_EXP_KARABINA
#define BLS_EXP_KARABINA 1
#endif
BLS_HD BLS_INLINE void fp12_cyc_exp_xabs(fp12& r, const fp12& a_in) {
#if BLS_EXP_KARABINA
  fp12_cyc_exp_xabs_karabina(r, a_in);
#else
  fp12_cyc_exp_xabs_gs(r, a_in);
#endif
}

BLS_HD BLS_CALL void final_exponentiation(fp12& r, const fp12& f_in) {
  const fp12 f = f_in;
  // easy part: f^((p^6-1)(p^2+1))
  fp12 t, fi, m;
  fp12_conj(t, f);
  fp12_inv(fi, f);
  BLS_FE_MUL(m, t, fi);
  fp12_frobenius(t, m, 2);
  BLS_FE_MUL(m, t, m);
  // hard part: m^((x-1)^2 (x+p)(x^2+p^2-1)) * m^3
  fp12 t0, t1, t2, u;
  // t0 = m^(x-1) = conj(m^|x| * m)
  fp12_cyc_exp_xabs(t0, m);
  BLS_FE_MUL(t0, t0, m);
  fp12_conj(t0, t0);
  // t0 = t0^(x-1)
  fp12_cyc_exp_xabs(u, t0);
  BLS_FE_MUL(u, u, t0);
  fp12_conj(t0, u);
  // t1 = t0^(x+p) = conj(t0^|x|) * frob(t0)
  fp12_cyc_exp_xabs(u, t0);
  fp12_conj(u, u);
  fp12_frobenius(t1, t0, 1);
  BLS_FE_MUL(t1, t1, u);
  // t2 = t1^(x^2+p^2-1) = (t1^|x|)^|x| * frob2(t1) * conj(t1)
  fp12_cyc_exp_xabs(u, t1);
  fp12_cyc_exp_xabs(u, u);
  fp12_frobenius(t2, t1, 2);
  BLS_FE_MUL(t2, t2, u);
  fp12_conj(u, t1);
  BLS_FE_MUL(t2, t2, u);
  // r = t2 * m^3
  fp12_cyclotomic_sqr(u, m);
  BLS_FE_MUL(u, u, m);
  BLS_FE_MUL(r, t2, u);
}

}  // namespace bls
