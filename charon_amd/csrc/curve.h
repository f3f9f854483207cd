// G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+u) over Fp2) group arithmetic,
// ZCash-format (de)compression and the fast subgroup tests, written once over a field type F
// (fp or fp2) via overloads.  Jacobian coordinates; the point at infinity has Z = 0.
//
// Serialization semantics follow herumi's ETH mode as pinned by the reference KATs
// (tests/golden/kat_reference.json) and oracle/bls12381.py::EDGE_POLICY.
#pragma once
#include "tower.h"

namespace bls {

// ---- field-generic overload set -----------------------------------------------------------
BLS_HD BLS_INLINE void f_add(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
BLS_HD BLS_INLINE void f_sub(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
BLS_HD BLS_INLINE void f_neg(fp& r, const fp& a) { fp_neg(r, a); }
BLS_HD BLS_INLINE void f_mul(fp& r, const fp& a, const fp& b) { fp_mul(r, a, b); }
BLS_HD BLS_INLINE void f_sqr(fp& r, const fp& a) { fp_sqr(r, a); }
BLS_HD BLS_INLINE bool f_is_zero(const fp& a) { return fp_is_zero(a); }
BLS_HD BLS_INLINE bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
BLS_HD BLS_INLINE void f_set_zero(fp& r) { fp_set_zero(r); }
BLS_HD BLS_INLINE void f_set_one(fp& r) { fp_set_one(r); }
BLS_HD BLS_INLINE void f_inv(fp& r, const fp& a) { fp_inv(r, a); }

BLS_HD BLS_INLINE void f_add(fp2& r, const fp2& a, const fp2& b) { fp2_add(r, a, b); }
BLS_HD BLS_INLINE void f_sub(fp2& r, const fp2& a, const fp2& b) { fp2_sub(r, a, b); }
BLS_HD BLS_INLINE void f_neg(fp2& r, const fp2& a) { fp2_neg(r, a); }
BLS_HD BLS_INLINE void f_mul(fp2& r, const fp2& a, const fp2& b) { fp2_mul(r, a, b); }
BLS_HD BLS_INLINE void f_sqr(fp2& r, const fp2& a) { fp2_sqr(r, a); }
BLS_HD BLS_INLINE bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
BLS_HD BLS_INLINE bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
BLS_HD BLS_INLINE void f_set_zero(fp2& r) { fp2_set_zero(r); }
BLS_HD BLS_INLINE void f_set_one(fp2& r) { fp2_set_one(r); }
BLS_HD BLS_INLINE void f_inv(fp2& r, const fp2& a) { fp2_inv(r, a); }

template <class F>
struct jac {
  F x, y, z;
};
template <class F>
struct aff {
  F x, y;
};
using g1j = jac<fp>;
using g2j = jac<fp2>;
using g1a = aff<fp>;
using g2a = aff<fp2>;

template <class F>
BLS_HD BLS_INLINE void jac_set_inf(jac<F>& r) {
  f_set_one(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
}
template <class F>
BLS_HD BLS_INLINE bool jac_is_inf(const jac<F>& a) {
  return f_is_zero(a.z);
}
template <class F>
BLS_HD BLS_INLINE void jac_from_aff(jac<F>& r, const aff<F>& a) {
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
}
template <class F>
BLS_HD BLS_INLINE void jac_neg(jac<F>& r, const jac<F>& a) {
  r.x = a.x;
  f_neg(r.y, a.y);
  r.z = a.z;
}

// dbl-2009-l (a = 0).  The body is force-inlined into the scalar-multiplication loops (the accumulator then stays
// in registers across doublings); jac_dbl is the called form for everything else.
template <class F>
BLS_HD BLS_INLINE void jac_dbl_body(jac<F>& r, const jac<F>& p) {
  F A, B, C, D, E, Fv, t;
  f_sqr(A, p.x);
  f_sqr(B, p.y);
  f_sqr(C, B);
  f_add(t, p.x, B);
  f_sqr(t, t);
  f_sub(t, t, A);
  f_sub(t, t, C);
  f_add(D, t, t);
  f_add(E, A, A);
  f_add(E, E, A);
  f_sqr(Fv, E);
  F z3;
  f_mul(z3, p.y, p.z);
  f_add(r.z, z3, z3);
  F x3;
  f_sub(x3, Fv, D);
  f_sub(x3, x3, D);
  f_sub(t, D, x3);
  f_mul(t, E, t);
  f_add(C, C, C);
  f_add(C, C, C);
  f_add(C, C, C);
  f_sub(r.y, t, C);
  r.x = x3;
}
template <class F>
BLS_HD BLS_CALL void jac_dbl(jac<F>& r, const jac<F>& p_in) {
  const jac<F> p = p_in;
  jac<F> t;
  jac_dbl_body(t, p);
  r = t;
}

// add-2007-bl with the exceptional cases handled (P = Q doubles, P = -Q gives infinity).  The _body form inlines into
// a loop (the MSM bucket and fold lanes, where a call would save and restore the live accumulators through scratch
// on every addition); jac_add is the out-of-line call everything else uses.
template <class F>
BLS_HD BLS_INLINE void jac_add_body(jac<F>& r, const jac<F>& p_in, const jac<F>& q_in) {
  const jac<F> p = p_in;
  const jac<F> q = q_in;
  if (jac_is_inf(p)) {
    r = q;
    return;
  }
  if (jac_is_inf(q)) {
    r = p;
    return;
  }
  F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  f_sqr(z1z1, p.z);
  f_sqr(z2z2, q.z);
  f_mul(u1, p.x, z2z2);
  f_mul(u2, q.x, z1z1);
  f_mul(s1, p.y, q.z);
  f_mul(s1, s1, z2z2);
  f_mul(s2, q.y, p.z);
  f_mul(s2, s2, z1z1);
  f_sub(h, u2, u1);
  f_sub(rr, s2, s1);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_add(rr, rr, rr);
  f_add(i, h, h);
  f_sqr(i, i);
  f_mul(j, h, i);
  f_mul(v, u1, i);
  F x3, y3, z3;
  f_sqr(x3, rr);
  f_sub(x3, x3, j);
  f_sub(x3, x3, v);
  f_sub(x3, x3, v);
  f_sub(t, v, x3);
  f_mul(y3, rr, t);
  f_mul(t, s1, j);
  f_add(t, t, t);
  f_sub(y3, y3, t);
  f_add(z3, p.z, q.z);
  f_sqr(z3, z3);
  f_sub(z3, z3, z1z1);
  f_sub(z3, z3, z2z2);
  f_mul(z3, z3, h);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

template <class F>
BLS_HD BLS_CALL void jac_add(jac<F>& r, const jac<F>& p_in, const jac<F>& q_in) {
  jac_add_body(r, p_in, q_in);
}

// mixed addition r = p + q with q affine (madd-2007-bl), exceptional cases handled (_body: inlined, as jac_add_body)
template <class F>
BLS_HD BLS_INLINE void jac_add_aff_body(jac<F>& r, const jac<F>& p_in, const aff<F>& q_in) {
  const jac<F> p = p_in;
  const aff<F> q = q_in;
  if (jac_is_inf(p)) {
    jac_from_aff(r, q);
    return;
  }
  F z1z1, u2, s2, h, hh, i, j, rr, v, t;
  f_sqr(z1z1, p.z);
  f_mul(u2, q.x, z1z1);
  f_mul(s2, q.y, p.z);
  f_mul(s2, s2, z1z1);
  f_sub(h, u2, p.x);
  f_sub(rr, s2, p.y);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_add(rr, rr, rr);
  f_sqr(hh, h);
  f_add(i, hh, hh);
  f_add(i, i, i);
  f_mul(j, h, i);
  f_mul(v, p.x, i);
  F x3, y3, z3;
  f_sqr(x3, rr);
  f_sub(x3, x3, j);
  f_sub(x3, x3, v);
  f_sub(x3, x3, v);
  f_sub(t, v, x3);
  f_mul(y3, rr, t);
  f_mul(t, p.y, j);
  f_add(t, t, t);
  f_sub(y3, y3, t);
  f_add(z3, p.z, h);
  f_sqr(z3, z3);
  f_sub(z3, z3, z1z1);
  f_sub(z3, z3, hh);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}
template <class F>
BLS_HD BLS_CALL void jac_add_aff(jac<F>& r, const jac<F>& p_in, const aff<F>& q_in) {
  jac_add_aff_body(r, p_in, q_in);
}

// r = [k] p for a 64-bit scalar k (uniform across lanes when k is a constant)
template <class F>
BLS_HD BLS_CALL void jac_mul_u64(jac<F>& r, const jac<F>& p_in, uint64_t k) {
  // Left-to-right from the top set bit (k is wave-uniform).  The doubling is inlined and the accumulator's address
  // is never taken, so it stays in registers; the base is read from the caller's frame by the few additions.
  jac<F> acc;
  jac_set_inf(acc);
  int i = 63;
  while (i >= 0 && !((k >> i) & 1ull)) --i;
  if (i >= 0) {
    acc = p_in;
    for (--i; i >= 0; --i) {
      jac<F> t;
      jac_dbl_body(t, acc);
      acc = t;
      if ((k >> i) & 1ull) {
        jac<F> x = acc, y;
        jac_add_body(y, x, p_in);  // inlined (one copy per field type): no scratch round trip per addition
        acc = y;
      }
    }
  }
  r = acc;
}

// r = [k] p for a scalar given as nlimbs little-endian 32-bit limbs
template <class F>
BLS_HD BLS_CALL void jac_mul_limbs(jac<F>& r, const jac<F>& p_in, const uint32_t* k, int nlimbs) {
  jac<F> acc;  // register-resident accumulator, inlined doubling (see jac_mul_u64)
  jac_set_inf(acc);
  for (int i = nlimbs * 32 - 1; i >= 0; --i) {
    jac<F> t;
    jac_dbl_body(t, acc);
    acc = t;
    if ((k[i >> 5] >> (i & 31)) & 1u) {
      jac<F> x = acc, y;
      jac_add_body(y, x, p_in);
      acc = y;
    }
  }
  r = acc;
}

// Jacobian equality without normalization
template <class F>
BLS_HD BLS_CALL bool jac_eq(const jac<F>& p_in, const jac<F>& q_in) {
  const jac<F> p = p_in;
  const jac<F> q = q_in;
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b;
  f_sqr(z1z1, p.z);
  f_sqr(z2z2, q.z);
  f_mul(a, p.x, z2z2);
  f_mul(b, q.x, z1z1);
  if (!f_eq(a, b)) return false;
  f_mul(a, p.y, q.z);
  f_mul(a, a, z2z2);
  f_mul(b, q.y, p.z);
  f_mul(b, b, z1z1);
  return f_eq(a, b);
}

template <class F>
BLS_HD BLS_CALL void jac_to_aff(aff<F>& r, const jac<F>& p_in) {
  const jac<F> p = p_in;
  F zi, zi2;
  f_inv(zi, p.z);
  f_sqr(zi2, zi);
  f_mul(r.x, p.x, zi2);
  f_mul(zi2, zi2, zi);
  f_mul(r.y, p.y, zi2);
}

BLS_HD BLS_INLINE bool aff_on_curve(const g1a& a) {
  fp l, r;
  fp_sqr(l, a.y);
  fp_sqr(r, a.x);
  fp_mul(r, r, a.x);
  fp_add(r, r, FP_B1);
  return fp_eq(l, r);
}
BLS_HD BLS_INLINE bool aff_on_curve(const g2a& a) {
  fp2 l, r;
  fp2_sqr(l, a.y);
  fp2_sqr(r, a.x);
  fp2_mul(r, r, a.x);
  fp2_add(r, r, FP2_B2);
  return fp2_eq(l, r);
}

// ---- endomorphisms --------------------------------------------------------------------------
// psi(x, y) = (conj(x) cx, conj(y) cy) on E'(Fp2); on Jacobian coordinates Z is conjugated too.
BLS_HD BLS_INLINE void g2_psi(g2j& r, const g2j& p) {
  fp2 t;
  fp2_conj(t, p.x);
  fp2_mul(r.x, t, PSI_CX);
  fp2_conj(t, p.y);
  fp2_mul(r.y, t, PSI_CY);
  fp2_conj(r.z, p.z);
}
BLS_HD BLS_INLINE void g2_psi2(g2j& r, const g2j& p) {
  fp2_mul(r.x, p.x, PSI2_CX);
  fp2_mul(r.y, p.y, PSI2_CY);
  r.z = p.z;
}

// P in G1  <=>  phi(P) = [-x^2] P   (Bowe 2019; beta chosen by tools/gen_constants.py)
// P in G2  <=>  psi(P) = [x] P      (Scott 2021)
// RFC 9380 G.3: h_eff * P via psi

// ---- (de)compression ------------------------------------------------------------------------
enum : int { DEC_OK = 0, DEC_BAD = 1, DEC_INF = 2 };

// Fp2 square root (complex method, one exponentiation to (p+1)/4 for the norm, one for the
// half-trace, one inversion).  Returns false when a is not a square.

// lexicographic "y > -y" used by the ZCash sign flag; y in Montgomery form
BLS_HD BLS_INLINE bool fp_is_lex_largest(const fp& y) {
  fp t;
  fp_from_mont(t, y);
  return fp_plain_gt_half(t);
}
BLS_HD BLS_INLINE bool fp2_is_lex_largest(const fp2& y) {
  fp t1;
  fp_from_mont(t1, y.c1);
  if (!fp_is_zero(t1)) return fp_plain_gt_half(t1);
  fp t0;
  fp_from_mont(t0, y.c0);
  return fp_plain_gt_half(t0);
}

// 48-byte compressed G1 -> affine; returns DEC_OK / DEC_BAD / DEC_INF.  Subgroup test included.

BLS_HD BLS_CALL bool g1_in_subgroup(const g1j& p_in) {
  const g1j p = p_in;
  if (jac_is_inf(p)) return true;
  g1j q;
  jac_mul_u64(q, p, X_ABS);
  jac_mul_u64(q, q, X_ABS);  // [x^2] P
  g1j phi;
  fp_mul(phi.x, p.x, FP_BETA);
  fp_neg(phi.y, p.y);  // -phi(P) compared with [x^2]P  <=>  phi(P) = [-x^2]P
  phi.z = p.z;
  return jac_eq(q, phi);
}
BLS_HD BLS_CALL bool g2_in_subgroup(const g2j& p_in) {
  const g2j p = p_in;
  if (jac_is_inf(p)) return true;
  g2j q, ps;
  jac_mul_u64(q, p, X_ABS);
  jac_neg(q, q);  // [x] P, x < 0
  g2_psi(ps, p);
  return jac_eq(q, ps);
}
BLS_HD BLS_CALL void g2_clear_cofactor(g2j& r, const g2j& p_in) {
  const g2j p = p_in;
  g2j t1, t2, t3, np;
  jac_mul_u64(t1, p, X_ABS);
  jac_neg(t1, t1);  // t1 = [x] P
  g2_psi(t2, p);    // t2 = psi(P)
  jac_dbl(t3, p);
  g2_psi2(t3, t3);  // t3 = psi^2(2P)
  g2j nt2;
  jac_neg(nt2, t2);
  jac_add(t3, t3, nt2);  // t3 = psi^2(2P) - psi(P)
  jac_add(t2, t1, t2);   // t2 = [x]P + psi(P)
  jac_mul_u64(t2, t2, X_ABS);
  jac_neg(t2, t2);       // t2 = [x] t2
  jac_add(t3, t3, t2);
  g2j nt1;
  jac_neg(nt1, t1);
  jac_add(t3, t3, nt1);
  jac_neg(np, p);
  jac_add(r, t3, np);
}

// k (8 little-endian limbs, k < 2^256) -> k / |x| in place; returns k mod |x|.  Bitwise long
// division: 256 shift-subtract steps on a 64-bit remainder (|x| < 2^64; when the remainder's top
// bit is set, 2*rem + b exceeds |x| and the wrapped difference is exact).
BLS_HD BLS_INLINE uint64_t u256_divmod_xabs(uint32_t* k) {
  uint64_t rem = 0;
  for (int w = 7; w >= 0; --w) {
    uint32_t q = 0;
    for (int b = 31; b >= 0; --b) {
      const uint64_t top = rem >> 63;
      rem = (rem << 1) | ((k[w] >> b) & 1u);
      if (top || rem >= X_ABS) {
        rem -= X_ABS;
        q |= 1u << b;
      }
    }
    k[w] = q;
  }
  return rem;
}

// r = [k] P for P in G2 (subgroup-checked) and a plain scalar k < r, 4-dimensional GLS split.
// On G2, psi = [x] and x = -|x|, so with k = e0 + e1|x| + e2|x|^2 + e3|x|^3 (base-|x| digits,
// r < |x|^4) [k]P = sum_i e_i (-psi)^i(P): 64 doublings and <= 64 additions over a 16-entry
// subset-sum table instead of a 255-bit double-and-add.
BLS_HD BLS_CALL void g2_mul_glv4(g2j& r, const g2j& p_in, const uint32_t* k_plain) {
  const g2j p = p_in;
  uint32_t k[8];
  for (int i = 0; i < 8; ++i) k[i] = k_plain[i];
  uint64_t e[4];
  for (int i = 0; i < 3; ++i) e[i] = u256_divmod_xabs(k);
  e[3] = (uint64_t)k[0] | ((uint64_t)k[1] << 32);
  g2j tab[16];
  jac_set_inf(tab[0]);
  tab[1] = p;                   // P
  g2_psi(tab[2], tab[1]);
  jac_neg(tab[2], tab[2]);      // -psi(P)
  g2_psi2(tab[4], tab[1]);      // psi^2(P)
  g2_psi(tab[8], tab[4]);
  jac_neg(tab[8], tab[8]);      // -psi^3(P)
  for (int d = 3; d < 16; ++d) {
    const int low = d & -d;
    if (d != low) jac_add(tab[d], tab[d ^ low], tab[low]);
  }
  g2j acc;
  jac_set_inf(acc);
  for (int bit = 63; bit >= 0; --bit) {
    g2j t;
    jac_dbl_body(t, acc);  // inlined; acc's address is never taken (it stays in registers)
    acc = t;
    const int d = (int)((e[0] >> bit) & 1u) | (int)(((e[1] >> bit) & 1u) << 1) |
                  (int)(((e[2] >> bit) & 1u) << 2) | (int)(((e[3] >> bit) & 1u) << 3);
    if (d) {
      g2j x = acc, y;
      jac_add(y, x, tab[d]);
      acc = y;
    }
  }
  r = acc;
}

// Second half of fp2_sqrt: given s with s^2 = N(a) = a0^2 + a1^2 (either sign), r = a square root of a; returns
// whether r^2 == a.  Split out so hash_to_g2 can share the norm's root between its two SSWU candidates.
BLS_HD BLS_CALL bool fp2_sqrt_from_norm_root(fp2& r, const fp2& a_in, const fp& s_in) {
  const fp2 a = a_in;
  const fp s = s_in;
  // a = a0 + a1 u: t = (a0 + s)/2, then sqrt(a) = x0 + a1/(2 x0) u with x0^2 = t, or a1/(2 x0) + x0 u with
  // x0^2 = -t when t is not a square.  One power z = t^((p-3)/4) gives both x0 = t z and 1/x0 = z (t square)
  // or -z (t^((p-1)/2) = -1).
  fp t, z, x0, inv_x0, t2;
  fp_add(t, a.c0, s);
  fp_mul(t, t, FP_HALF);
  if (fp_is_zero(t)) t = a.c0;  // a1 = 0 and s = -a0: use s = a0 instead
  fp_pow(z, t, EXP_SQRT_M1, 378);
  fp_mul(x0, z, t);
  fp_sqr(t2, x0);
  const bool t_square = fp_eq(t2, t);
  if (t_square)
    inv_x0 = z;
  else
    fp_neg(inv_x0, z);
  fp y0, y1;
  fp_mul(y1, a.c1, inv_x0);
  fp_mul(y1, y1, FP_HALF);  // a1 / (2 x0)
  if (t_square) {
    y0 = x0;
  } else {
    y0 = y1;
    y1 = x0;
  }
  fp2 cand;
  cand.c0 = y0;
  cand.c1 = y1;
  fp2 chk;
  fp2_sqr(chk, cand);
  r = cand;
  return fp2_eq(chk, a);
}

BLS_HD BLS_CALL bool fp2_sqrt(fp2& r, const fp2& a_in) {
  const fp2 a = a_in;
  fp n, s, t;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  fp_sqrt(s, n);  // candidate; correctness is checked at the end
  return fp2_sqrt_from_norm_root(r, a, s);
}

BLS_HD BLS_CALL int g1_decompress(g1a& out, const uint8_t* b, bool subgroup_check) {
  const uint8_t flags = b[0];
  if (!(flags & 0x80)) return DEC_BAD;
  uint8_t buf[48];
  for (int i = 0; i < 48; ++i) buf[i] = b[i];
  buf[0] &= 0x1f;
  if (flags & 0x40) {
    uint8_t acc = flags & 0x20;
    for (int i = 0; i < 48; ++i) acc |= buf[i];
    return acc ? DEC_BAD : DEC_INF;
  }
  fp x;
  fp_plain_from_be48(x, buf);
  if (!fp_plain_lt_p(x)) return DEC_BAD;
  fp_to_mont(x, x);
  fp y2, y;
  fp_sqr(y2, x);
  fp_mul(y2, y2, x);
  fp_add(y2, y2, FP_B1);
  if (!fp_sqrt(y, y2)) return DEC_BAD;
  if (fp_is_lex_largest(y) != ((flags & 0x20) != 0)) fp_neg(y, y);
  out.x = x;
  out.y = y;
  if (subgroup_check) {
    g1j pj;
    jac_from_aff(pj, out);
    if (!g1_in_subgroup(pj)) return DEC_BAD;
  }
  return DEC_OK;
}

BLS_HD BLS_CALL int g2_decompress(g2a& out, const uint8_t* b, bool subgroup_check) {
  const uint8_t flags = b[0];
  if (!(flags & 0x80)) return DEC_BAD;
  uint8_t buf[96];
  for (int i = 0; i < 96; ++i) buf[i] = b[i];
  buf[0] &= 0x1f;
  if (flags & 0x40) {
    uint8_t acc = flags & 0x20;
    for (int i = 0; i < 96; ++i) acc |= buf[i];
    return acc ? DEC_BAD : DEC_INF;
  }
  fp2 x;
  fp_plain_from_be48(x.c1, buf);
  fp_plain_from_be48(x.c0, buf + 48);
  if (!fp_plain_lt_p(x.c0) || !fp_plain_lt_p(x.c1)) return DEC_BAD;
  fp_to_mont(x.c0, x.c0);
  fp_to_mont(x.c1, x.c1);
  fp2 y2, y;
  fp2_sqr(y2, x);
  fp2_mul(y2, y2, x);
  fp2_add(y2, y2, FP2_B2);
  if (!fp2_sqrt(y, y2)) return DEC_BAD;
  if (fp2_is_lex_largest(y) != ((flags & 0x20) != 0)) fp2_neg(y, y);
  out.x = x;
  out.y = y;
  if (subgroup_check) {
    g2j pj;
    jac_from_aff(pj, out);
    if (!g2_in_subgroup(pj)) return DEC_BAD;
  }
  return DEC_OK;
}

BLS_HD BLS_CALL void g1_compress(uint8_t* b, const g1j& p) {
  if (jac_is_inf(p)) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; ++i) b[i] = 0;
    return;
  }
  g1a a;
  jac_to_aff(a, p);
  fp x;
  fp_from_mont(x, a.x);
  fp_plain_to_be48(b, x);
  b[0] |= 0x80;
  if (fp_is_lex_largest(a.y)) b[0] |= 0x20;
}

BLS_HD BLS_CALL void g2_compress(uint8_t* b, const g2j& p) {
  if (jac_is_inf(p)) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; ++i) b[i] = 0;
    return;
  }
  g2a a;
  jac_to_aff(a, p);
  fp x1, x0;
  fp_from_mont(x1, a.x.c1);
  fp_from_mont(x0, a.x.c0);
  fp_plain_to_be48(b, x1);
  fp_plain_to_be48(b + 48, x0);
  b[0] |= 0x80;
  if (fp2_is_lex_largest(a.y)) b[0] |= 0x20;
}

}  // namespace bls
