// Extension tower for BLS12-381:  Fp2 = Fp[u]/(u^2+1),  Fp6 = Fp2[v]/(v^3-xi),  Fp12 = Fp6[w]/(w^2-v),
// xi = 1+u.  Same tower as the oracle (oracle/bls12381.py) so Fp12 values are comparable limb for
// limb, but the formulas here are the lane-local Karatsuba / sparse forms the kernels run.
#pragma once
#include "field.h"

// Fp6 products are inlined into the Fp12 functions (op_probe: fp12_sqr 227k -> 170k cycles, fp12_mul 319k -> 254k):
// across a real call their 72-dword operands and result travel through the stack.  -DBLS_FP6_CALL=BLS_CALL restores calls.
#ifndef BLS_FP6_CALL
#define BLS_FP6_CALL BLS_INLINE
#endif
// Miller-loop building blocks (Fp12 squaring, line products, doubling/addition steps) are inlined into the loop: no
// call boundary means no callee-saved register spills and no stack round trip of f, T and the lines per step
// (op_probe: miller_loop_n 42.7M -> 41.2M cycles; C2 +1.6 %).  -DBLS_MILLER_CALL=BLS_CALL restores calls.
#ifndef BLS_MILLER_CALL
#define BLS_MILLER_CALL BLS_INLINE
#endif

namespace bls {

struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------------------------- Fp2
BLS_HD BLS_INLINE void fp2_set_zero(fp2& r) {
  fp_set_zero(r.c0);
  fp_set_zero(r.c1);
}
BLS_HD BLS_INLINE void fp2_set_one(fp2& r) {
  fp_set_one(r.c0);
  fp_set_zero(r.c1);
}
BLS_HD BLS_INLINE bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BLS_HD BLS_INLINE bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BLS_HD BLS_INLINE void fp2_add(fp2& r, const fp2& a, const fp2& b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
BLS_HD BLS_INLINE void fp2_sub(fp2& r, const fp2& a, const fp2& b) {
  fp_sub(r.c0, a.c0, b.c0);
  fp_sub(r.c1, a.c1, b.c1);
}
BLS_HD BLS_INLINE void fp2_neg(fp2& r, const fp2& a) {
  fp_neg(r.c0, a.c0);
  fp_neg(r.c1, a.c1);
}
BLS_HD BLS_INLINE void fp2_dbl(fp2& r, const fp2& a) { fp2_add(r, a, a); }
BLS_HD BLS_INLINE void fp2_conj(fp2& r, const fp2& a) {
  r.c0 = a.c0;
  fp_neg(r.c1, a.c1);
}
#if defined(__HIP_DEVICE_COMPILE__) && BLS_FP2_PAIR
__device__ __forceinline__ void fp2p_join(fp2& r, const u32x12& c, uint32_t hm);
BLS_HD BLS_INLINE void fp2_mul_fp(fp2& r, const fp2& a, const fp& b) {  // one Fp product per lane (split-Fp2 build)
  const uint32_t hm = fp2p_mask();
  fp x, y;
#pragma unroll
  for (int j = 0; j < 12; ++j) x.v[j] = (hm & a.c1.v[j]) | (~hm & a.c0.v[j]);
  fp_mul(y, x, b);
  fp2p_join(r, fp_to_vec(y), hm);
}
#else
BLS_HD BLS_INLINE void fp2_mul_fp(fp2& r, const fp2& a, const fp& b) {
  fp_mul(r.c0, a.c0, b);
  fp_mul(r.c1, a.c1, b);
}
#endif
// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
BLS_HD BLS_INLINE void fp2_mul_xi(fp2& r, const fp2& a) {
  fp t;
  fp_sub(t, a.c0, a.c1);
  fp_add(r.c1, a.c0, a.c1);
  r.c0 = t;
}
BLS_HD BLS_INLINE void fp2_half(fp2& r, const fp2& a) {
  fp_half(r.c0, a.c0);
  fp_half(r.c1, a.c1);
}
// r = a * 3b' = a * 12 (1 + u) (the twist's 3b, b' = 4(1 + u)): additions only
BLS_HD BLS_INLINE void fp2_mul_3b2(fp2& r, const fp2& a) {
  fp2 t, t4;
  fp2_mul_xi(t, a);
  fp2_add(t, t, t);    // 2 xi a
  fp2_add(t4, t, t);   // 4 xi a
  fp2_add(t, t4, t4);  // 8 xi a
  fp2_add(r, t, t4);   // 12 xi a
}
BLS_HD BLS_INLINE void fp2_mul_small(fp2& r, const fp2& a, uint32_t k) {
  fp_mul_small(r.c0, a.c0, k);
  fp_mul_small(r.c1, a.c1, k);
}


// ---------------------------------------------------------------------------------- Fp6
BLS_HD BLS_INLINE void fp6_set_zero(fp6& r) {
  fp2_set_zero(r.c0);
  fp2_set_zero(r.c1);
  fp2_set_zero(r.c2);
}
BLS_HD BLS_INLINE void fp6_set_one(fp6& r) {
  fp2_set_one(r.c0);
  fp2_set_zero(r.c1);
  fp2_set_zero(r.c2);
}
BLS_HD BLS_INLINE void fp6_add(fp6& r, const fp6& a, const fp6& b) {
  fp2_add(r.c0, a.c0, b.c0);
  fp2_add(r.c1, a.c1, b.c1);
  fp2_add(r.c2, a.c2, b.c2);
}
BLS_HD BLS_INLINE void fp6_sub(fp6& r, const fp6& a, const fp6& b) {
  fp2_sub(r.c0, a.c0, b.c0);
  fp2_sub(r.c1, a.c1, b.c1);
  fp2_sub(r.c2, a.c2, b.c2);
}
BLS_HD BLS_INLINE void fp6_neg(fp6& r, const fp6& a) {
  fp2_neg(r.c0, a.c0);
  fp2_neg(r.c1, a.c1);
  fp2_neg(r.c2, a.c2);
}
// r = a * v
BLS_HD BLS_INLINE void fp6_mul_v(fp6& r, const fp6& a) {
  fp2 t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}
// r = a * (b0 + b1 v)
// r = a * (b1 v)

// ---------------------------------------------------------------------------------- Fp12
BLS_HD BLS_INLINE void fp12_set_one(fp12& r) {
  fp6_set_one(r.c0);
  fp6_set_zero(r.c1);
}
BLS_HD BLS_INLINE bool fp12_is_one(const fp12& a) {
  fp12 one;
  fp12_set_one(one);
  bool eq = true;
  const fp* x = &a.c0.c0.c0;
  const fp* y = &one.c0.c0.c0;
  for (int i = 0; i < 12; ++i) eq = eq && fp_eq(x[i], y[i]);
  return eq;
}
BLS_HD BLS_INLINE void fp12_conj(fp12& r, const fp12& a) {
  r.c0 = a.c0;
  fp6_neg(r.c1, a.c1);
}
// f *= line with the M-twist sparse shape (g0 + g1 v) + (h1 v) w
// Frobenius x -> x^(p^j), j in {1,2,3}
// Granger-Scott squaring for elements of the cyclotomic subgroup

#if defined(__HIP_DEVICE_COMPILE__) && BLS_FP2_PAIR
// Split-Fp2 build (field.h fp2p_*): this lane forms one coefficient (its half of gen_fp2_mul's two sums of products),
// the partner lane l ^ 4 the other, and one exchange gives both lanes the full, canonical product.
__device__ __forceinline__ void fp2p_join(fp2& r, const u32x12& c, uint32_t hm) {
  fp mine, other;
  fp_from_vec(mine, c);
#pragma unroll
  for (int j = 0; j < 12; ++j) other.v[j] = fp2p_xchg(mine.v[j]);
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    r.c0.v[j] = (hm & other.v[j]) | (~hm & mine.v[j]);
    r.c1.v[j] = (hm & mine.v[j]) | (~hm & other.v[j]);
  }
}
BLS_HD BLS_INLINE void fp2_mul(fp2& r, const fp2& a, const fp2& b) {
  u32x12 a0 = fp_to_vec(a.c0), a1 = fp_to_vec(a.c1), b0 = fp_to_vec(b.c0), b1 = fp_to_vec(b.c1), c;
  uint32_t hm = fp2p_mask();
  const uint32_t h = hm;
  asm volatile(BLS_ASM_CALL("bls_fp2_mul_half_rt")
               : "+{v[0:11]}"(a0), "+{v[12:23]}"(a1), "+{v[24:35]}"(b0), "+{v[36:47]}"(b1), "={v[52:63]}"(c),
                 "+{v76}"(hm)
               : BLS_P_SGPR_IN
               : BLS_FP2_MUL_HALF_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp2p_join(r, c, h);
}
BLS_HD BLS_INLINE void fp2_sqr(fp2& r, const fp2& a) {
  u32x12 a0 = fp_to_vec(a.c0), a1 = fp_to_vec(a.c1), c;
  uint32_t hm = fp2p_mask();
  const uint32_t h = hm;
  asm volatile(BLS_ASM_CALL("bls_fp2_sqr_half_rt")
               : "+{v[0:11]}"(a0), "+{v[12:23]}"(a1), "={v[24:35]}"(c), "+{v76}"(hm)
               : BLS_P_SGPR_IN
               : BLS_FP2_SQR_HALF_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp2p_join(r, c, h);
}
#elif defined(__HIP_DEVICE_COMPILE__)
// Device: one asm routine (tools/gen_fp_asm.py gen_fp2_mul): each coefficient is a single Montgomery reduction of
// a sum of two products, c1 = (a0 b1 + a1 b0)/R and c0 = (a0 b0 + a1 (2p - b1))/R -- no Fp additions and two final
// subtractions instead of Karatsuba's three reduced products, three subtractions and two sums.  Operands may be
// unreduced sums in [0, 2p) (fp2_add_lazy); the result is canonical.  (The routine leaves a0, a1, b0 intact, but
// declaring them input-only crashes this compiler's register allocator, so they are in/out operands here.)
BLS_HD BLS_INLINE void fp2_mul(fp2& r, const fp2& a, const fp2& b) {
  u32x12 a0 = fp_to_vec(a.c0), a1 = fp_to_vec(a.c1), b0 = fp_to_vec(b.c0), b1 = fp_to_vec(b.c1), c0, c1;
  asm volatile(BLS_ASM_CALL("bls_fp2_mul_rt")
               : "+{v[0:11]}"(a0), "+{v[12:23]}"(a1), "+{v[24:35]}"(b0), "+{v[36:47]}"(b1), "={v[52:63]}"(c1),
                 "={v[64:75]}"(c0)
               : BLS_P_SGPR_IN
               : BLS_FP2_MUL_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp_from_vec(r.c0, c0);
  fp_from_vec(r.c1, c1);
}
#else
BLS_HD BLS_INLINE void fp2_mul(fp2& r, const fp2& a_in, const fp2& b_in) {
  // Karatsuba: 3 Fp products; the two sums only feed the third product, so they stay unreduced (fp_add_lazy)
#if defined(BLS_CONTRACT_CHECK)
  // the device routine's operands: below 2^382 each, and 2p - b1 formed inside it (b1 <= 2p)
  BLS_CONTRACT(fp_product_operand(a_in.c0) && fp_product_operand(a_in.c1) && fp_product_operand(b_in.c0) &&
                   fp_product_operand(b_in.c1),
               "fp2_mul: an operand is not below 2p and 2^382");
  g_contract_lazy_operands += !fp_canonical(a_in.c0) || !fp_canonical(a_in.c1) || !fp_canonical(b_in.c0) ||
                              !fp_canonical(b_in.c1);
  fp2 a, b;
  fp_reduce_2p(a.c0, a_in.c0);
  fp_reduce_2p(a.c1, a_in.c1);
  fp_reduce_2p(b.c0, b_in.c0);
  fp_reduce_2p(b.c1, b_in.c1);
#else
  const fp2& a = a_in;
  const fp2& b = b_in;
#endif
  fp t0, t1, t2, s0, s1;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add_lazy(s0, a.c0, a.c1);
  fp_add_lazy(s1, b.c0, b.c1);
  fp_mul(t2, s0, s1);
  fp_sub(r.c0, t0, t1);
  fp_sub(t2, t2, t0);
  fp_sub(r.c1, t2, t1);
}
#endif
// Sums of Fp2 products with ONE Montgomery reduction per output coefficient (the lazy-reduction experiment,
// BLS_LAZY_FP6; tools/gen_fp_asm.py gen_fp2_mul2 / gen_fp2_mul3): r = x y + z w (+ u t).  Canonical operands.
#if defined(__HIP_DEVICE_COMPILE__) && BLS_LAZY_FP6 && !BLS_FP2_PAIR
BLS_HD BLS_INLINE void fp2_mul2(fp2& r, const fp2& x, const fp2& y, const fp2& z, const fp2& w) {
  u32x12 x0 = fp_to_vec(x.c0), x1 = fp_to_vec(x.c1), y0 = fp_to_vec(y.c0), y1 = fp_to_vec(y.c1);
  u32x12 z0 = fp_to_vec(z.c0), z1 = fp_to_vec(z.c1), w0 = fp_to_vec(w.c0), w1 = fp_to_vec(w.c1), c0, c1;
  asm volatile(BLS_ASM_CALL("bls_fp2_mul2_rt")
               : "+{v[0:11]}"(x0), "+{v[12:23]}"(x1), "+{v[24:35]}"(y0), "+{v[36:47]}"(y1), "+{v[88:99]}"(z0),
                 "+{v[100:111]}"(z1), "+{v[112:123]}"(w0), "+{v[124:135]}"(w1), "={v[52:63]}"(c1), "={v[64:75]}"(c0)
               :
               : BLS_FP2_MUL2_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp_from_vec(r.c0, c0);
  fp_from_vec(r.c1, c1);
}
BLS_HD BLS_INLINE void fp2_mul3(fp2& r, const fp2& x, const fp2& y, const fp2& z, const fp2& w, const fp2& u,
                                const fp2& t) {
  u32x12 x0 = fp_to_vec(x.c0), x1 = fp_to_vec(x.c1), y0 = fp_to_vec(y.c0), y1 = fp_to_vec(y.c1);
  u32x12 z0 = fp_to_vec(z.c0), z1 = fp_to_vec(z.c1), w0 = fp_to_vec(w.c0), w1 = fp_to_vec(w.c1);
  u32x12 u0 = fp_to_vec(u.c0), u1 = fp_to_vec(u.c1), t0 = fp_to_vec(t.c0), t1 = fp_to_vec(t.c1), c0, c1;
  asm volatile(BLS_ASM_CALL("bls_fp2_mul3_rt")
               : "+{v[0:11]}"(x0), "+{v[12:23]}"(x1), "+{v[24:35]}"(y0), "+{v[36:47]}"(y1), "+{v[88:99]}"(z0),
                 "+{v[100:111]}"(z1), "+{v[112:123]}"(w0), "+{v[124:135]}"(w1), "+{v[136:147]}"(u0),
                 "+{v[148:159]}"(u1), "+{v[160:171]}"(t0), "+{v[172:183]}"(t1), "={v[52:63]}"(c1), "={v[64:75]}"(c0)
               :
               : BLS_FP2_MUL2_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp_from_vec(r.c0, c0);
  fp_from_vec(r.c1, c1);
}
#else
BLS_HD BLS_INLINE void fp2_mul2(fp2& r, const fp2& x, const fp2& y, const fp2& z, const fp2& w) {
  fp2 a, b;
  fp2_mul(a, x, y);
  fp2_mul(b, z, w);
  fp2_add(r, a, b);
}
BLS_HD BLS_INLINE void fp2_mul3(fp2& r, const fp2& x, const fp2& y, const fp2& z, const fp2& w, const fp2& u,
                                const fp2& t) {
  fp2 a, b;
  fp2_mul2(a, x, y, z, w);
  fp2_mul(b, u, t);
  fp2_add(r, a, b);
}
#endif
// (a0+a1)(a0-a1) + 2 a0 a1 u with three Fp products; the sum and difference only feed the product: unreduced
BLS_HD BLS_INLINE void fp2_sqr_c(fp2& r, const fp2& a) {
  fp s, d, m;
  fp_add_lazy(s, a.c0, a.c1);
  fp_sub_lazy(d, a.c0, a.c1);
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
}
#if defined(__HIP_DEVICE_COMPILE__) && BLS_FP2_PAIR
// (split-Fp2 fp2_sqr above)
#elif defined(__HIP_DEVICE_COMPILE__)
// Device: one asm routine (tools/gen_fp_asm.py gen_fp2_sqr): c0 = (a0+a1)(a0+p-a1)/R, c1 = a0 (2 a1)/R with the three
// operand sums unreduced inside it.
BLS_HD BLS_INLINE void fp2_sqr(fp2& r, const fp2& a) {
  u32x12 a0 = fp_to_vec(a.c0), a1 = fp_to_vec(a.c1), c0, c1;
  asm volatile(BLS_ASM_CALL("bls_fp2_sqr_rt")
               : "+{v[0:11]}"(a0), "+{v[12:23]}"(a1), "={v[24:35]}"(c0), "={v[36:47]}"(c1)
               : BLS_P_SGPR_IN
               : BLS_FP2_SQR_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
  fp_from_vec(r.c0, c0);
  fp_from_vec(r.c1, c1);
}
#else
BLS_HD BLS_INLINE void fp2_sqr(fp2& r, const fp2& a) {
  // the device routine forms (a0 + a1), (a0 + p - a1) and 2 a1 inside it: canonical operands only
  BLS_CONTRACT(fp_canonical(a.c0) && fp_canonical(a.c1), "fp2_sqr: an operand is not canonical");
  fp2_sqr_c(r, a);
}
#endif
// The cyclotomic squaring's Fp2 squarings use the three-product C form: inside the inlined exponentiation loop the
// routine's 64 pinned registers cost more spills than it saves (op_probe: fp12_cyc_exp_xabs 5.86M -> 5.64M cycles).
#ifndef BLS_CYC_FP2_SQR
#if BLS_FP2_PAIR
#define BLS_CYC_FP2_SQR fp2_sqr
#else
#define BLS_CYC_FP2_SQR fp2_sqr_c
#endif
#endif
BLS_HD BLS_CALL void fp2_inv(fp2& r, const fp2& a_in) {
  const fp2 a = a_in;
  fp t0, t1;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(t0, t0, t1);
  fp_inv(t1, t0);
  fp_mul(r.c0, a.c0, t1);
  fp_mul(t0, a.c1, t1);
  fp_neg(r.c1, t0);
}

// a + b left unreduced in [0, 2p) for canonical a, b: only ever an operand of fp2_mul (device), which reduces it.
BLS_HD BLS_INLINE void fp2_add_lazy(fp2& r, const fp2& a, const fp2& b) {
  fp_add_lazy(r.c0, a.c0, b.c0);
  fp_add_lazy(r.c1, a.c1, b.c1);
}

BLS_HD BLS_FP6_CALL void fp6_mul(fp6& r, const fp6& a_in, const fp6& b_in) {
  // Karatsuba over Fp2 (6 Fp2 products); a, b canonical.  Operands are copied in once: referenced operands live in
  // the caller's frame, and re-reading them around every product exposes a flat-load round trip each time.  The
  // Karatsuba sums only feed products, so they stay unreduced.
  const fp6 a = a_in, b = b_in;
  fp2 t0, t1, t2, s0, s1, u0, u1, u2;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  fp2_add_lazy(s0, a.c1, a.c2);
  fp2_add_lazy(s1, b.c1, b.c2);
  fp2_mul(u0, s0, s1);
  fp2_sub(u0, u0, t1);
  fp2_sub(u0, u0, t2);
  fp2_mul_xi(u0, u0);
  fp2_add(u0, u0, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fp2_add_lazy(s0, a.c0, a.c1);
  fp2_add_lazy(s1, b.c0, b.c1);
  fp2_mul(u1, s0, s1);
  fp2_sub(u1, u1, t0);
  fp2_sub(u1, u1, t1);
  fp2 x2;
  fp2_mul_xi(x2, t2);
  fp2_add(u1, u1, x2);
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fp2_add_lazy(s0, a.c0, a.c2);
  fp2_add_lazy(s1, b.c0, b.c2);
  fp2_mul(u2, s0, s1);
  fp2_sub(u2, u2, t0);
  fp2_sub(u2, u2, t2);
  fp2_add(u2, u2, t1);
  r.c0 = u0;
  r.c1 = u1;
  r.c2 = u2;
}
BLS_HD BLS_FP6_CALL void fp6_sqr(fp6& r, const fp6& a_in) {
  const fp6 a = a_in;
  // Chung-Hasan SQR2
  fp2 s0, s1, s2, s3, s4, t;
  fp2_sqr(s0, a.c0);
  fp2_mul(s1, a.c0, a.c1);
  fp2_dbl(s1, s1);
  fp2_sub(t, a.c0, a.c1);
  fp2_add(t, t, a.c2);
  fp2_sqr(s2, t);
  fp2_mul(s3, a.c1, a.c2);
  fp2_dbl(s3, s3);
  fp2_sqr(s4, a.c2);
  fp2 c0, c1, c2;
  fp2_mul_xi(c0, s3);
  fp2_add(c0, c0, s0);
  fp2_mul_xi(c1, s4);
  fp2_add(c1, c1, s1);
  fp2_add(c2, s1, s2);
  fp2_add(c2, c2, s3);
  fp2_sub(c2, c2, s0);
  fp2_sub(c2, c2, s4);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
BLS_HD BLS_CALL void fp6_inv(fp6& r, const fp6& a_in) {
  const fp6 a = a_in;
  fp2 c0, c1, c2, t, s;
  fp2_sqr(c0, a.c0);
  fp2_mul(t, a.c1, a.c2);
  fp2_mul_xi(t, t);
  fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2);
  fp2_mul_xi(c1, c1);
  fp2_mul(t, a.c0, a.c1);
  fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1);
  fp2_mul(t, a.c0, a.c2);
  fp2_sub(c2, c2, t);
  fp2_mul(t, a.c2, c1);
  fp2_mul(s, a.c1, c2);
  fp2_add(t, t, s);
  fp2_mul_xi(t, t);
  fp2_mul(s, a.c0, c0);
  fp2_add(t, t, s);
  fp2_inv(t, t);
  fp2_mul(r.c0, c0, t);
  fp2_mul(r.c1, c1, t);
  fp2_mul(r.c2, c2, t);
}
BLS_HD BLS_FP6_CALL void fp6_mul_01(fp6& r, const fp6& a_in, const fp2& b0_in, const fp2& b1_in) {
  const fp6 a = a_in;
  const fp2 b0 = b0_in;
  const fp2 b1 = b1_in;
  // (a0 + a1 v + a2 v^2)(b0 + b1 v): 5 Fp2 products
  fp2 t0, t1, s0, s1, u;
  fp2_mul(t0, a.c0, b0);
  fp2_mul(t1, a.c1, b1);
  fp2 c0, c1, c2;
  // c0 = t0 + xi * a2 b1
  fp2_mul(u, a.c2, b1);
  fp2_mul_xi(u, u);
  fp2_add(c0, u, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1
  fp2_add_lazy(s0, a.c0, a.c1);
  fp2_add(s1, b0, b1);  // full: b1 may itself be a sum (fp12_mul_line's g1 + h1)
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);
  // c2 = a2 b0 + t1
  fp2_mul(c2, a.c2, b0);
  fp2_add(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
BLS_HD BLS_FP6_CALL void fp6_mul_1(fp6& r, const fp6& a_in, const fp2& b1_in) {
  const fp6 a = a_in;
  const fp2 b1 = b1_in;
  // (a0 + a1 v + a2 v^2) b1 v = xi a2 b1 + a0 b1 v + a1 b1 v^2
  fp2 c0, c1, c2;
  fp2_mul(c0, a.c2, b1);
  fp2_mul_xi(c0, c0);
  fp2_mul(c1, a.c0, b1);
  fp2_mul(c2, a.c1, b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}

// Operands read where they are needed rather than copied in at entry: the 288-dword copy made the allocator spill
// (op_probe: fp12_mul 242k -> 218k cycles, final_exponentiation -3.5 %).
#ifndef BLS_FP12_MUL_COPYIN
#define BLS_FP12_MUL_COPYIN 0
#endif
BLS_HD BLS_INLINE void fp12_mul_inl(fp12& r, const fp12& a_in, const fp12& b_in) {
#if BLS_FP12_MUL_COPYIN
  const fp12 a = a_in;
  const fp12 b = b_in;
#else
  const fp12& a = a_in;
  const fp12& b = b_in;
#endif
  fp6 t0, t1, s0, s1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6 c1;
  fp6_mul(c1, s0, s1);
  fp6_sub(c1, c1, t0);
  fp6_sub(c1, c1, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
  r.c1 = c1;
}
BLS_HD BLS_CALL void fp12_mul(fp12& r, const fp12& a_in, const fp12& b_in) { fp12_mul_inl(r, a_in, b_in); }
BLS_HD BLS_INLINE void fp12_sqr_inl(fp12& r, const fp12& a_in) {
  // complex squaring: c0 = (a0+a1)(a0+v a1) - t - v t, c1 = 2t, t = a0 a1
  const fp12 a = a_in;
  fp6 t, s0, s1, vt;
  fp6_mul(t, a.c0, a.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_mul_v(s1, a.c1);
  fp6_add(s1, s1, a.c0);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t);
  fp6_mul_v(vt, t);
  fp6_sub(r.c0, s0, vt);
  fp6_add(r.c1, t, t);
}
BLS_HD BLS_MILLER_CALL void fp12_sqr(fp12& r, const fp12& a_in) { fp12_sqr_inl(r, a_in); }
BLS_HD BLS_CALL void fp12_inv(fp12& r, const fp12& a_in) {
  const fp12 a = a_in;
  fp6 t0, t1;
  fp6_sqr(t0, a.c0);
  fp6_sqr(t1, a.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t0, t0);
  fp6_mul(r.c0, a.c0, t0);
  fp6_mul(t1, a.c1, t0);
  fp6_neg(r.c1, t1);
}
BLS_HD BLS_MILLER_CALL void fp12_mul_line(fp12& f_in, const fp2& g0_in, const fp2& g1_in, const fp2& h1_in) {
  const fp2 g0 = g0_in;
  const fp2 g1 = g1_in;
  const fp2 h1 = h1_in;
  fp12 f = f_in;
  // f = (a0 + a1 w)(G + H w), G = g0 + g1 v, H = h1 v:
  //   c0 = a0 G + v (a1 H),  c1 = (a0 + a1)(G + H) - a0 G - a1 H
  fp6 t0, t1, s;
  fp6_mul_01(t0, f.c0, g0, g1);
  fp6_mul_1(t1, f.c1, h1);
  fp6_add(s, f.c0, f.c1);
  fp2 gh1;
  fp2_add(gh1, g1, h1);
  fp6_mul_01(s, s, g0, gh1);
  fp6_sub(s, s, t0);
  fp6_sub(f.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(f.c0, t0, t1);
  f_in = f;
}
// f *= la * lb for two M-twist lines l = (g0 + g1 v) + (h1 v) w.  The line product is
// (c0 dense) + (x v + y v^2) w with w^2 = v, v^3 = xi (6 Fp2 products); multiplying it into f
// costs 17 more, 23 in all instead of 26 for two fp12_mul_line calls.
BLS_HD BLS_INLINE void fp12_mul_line2_inl(fp12& f_in, const fp2& ga0_in, const fp2& ga1_in, const fp2& ha1_in, const fp2& gb0_in,
                                    const fp2& gb1_in, const fp2& hb1_in) {
  const fp2 ga0 = ga0_in;
  const fp2 ga1 = ga1_in;
  const fp2 ha1 = ha1_in;
  const fp2 gb0 = gb0_in;
  const fp2 gb1 = gb1_in;
  const fp2 hb1 = hb1_in;
  fp12 f = f_in;
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
  fp2_sub(L0.c1, t, p11);   // ga0 gb1 + ga1 gb0
  fp2_mul_xi(t, phh);
  fp2_add(L0.c0, p00, t);   // ga0 gb0 + xi ha1 hb1
  L0.c2 = p11;              // ga1 gb1
  fp2_add_lazy(sa, ga0, ha1);
  fp2_add_lazy(sb, gb0, hb1);
  fp2_mul(x, sa, sb);
  fp2_sub(x, x, p00);
  fp2_sub(x, x, phh);       // ga0 hb1 + ha1 gb0
  fp2_add_lazy(sa, ga1, ha1);
  fp2_add_lazy(sb, gb1, hb1);
  fp2_mul(y, sa, sb);
  fp2_sub(y, y, p11);
  fp2_sub(y, y, phh);       // ga1 hb1 + ha1 gb1
  // f = (F0 + F1 w)(L0 + L1 w), L1 = x v + y v^2
  fp6 t0, t1, s, l;
  fp6_mul(t0, f.c0, L0);
  {  // t1 = F1 * (x v + y v^2) = xi(a1 y + a2 x) + (a0 x + xi a2 y) v + (a0 y + a1 x) v^2
    const fp6& a = f.c1;
    fp2 m1, m2, m0, u, w2;
    fp2_mul(m1, a.c1, x);
    fp2_mul(m2, a.c2, y);
    fp2_mul(m0, a.c0, x);
    fp2_add_lazy(u, a.c1, a.c2);
    fp2_add_lazy(w2, x, y);
    fp2_mul(u, u, w2);
    fp2_sub(u, u, m1);
    fp2_sub(u, u, m2);
    fp2_mul_xi(t1.c0, u);
    fp2_mul_xi(u, m2);
    fp2_add(t1.c1, m0, u);
    fp2_mul(u, a.c0, y);
    fp2_add(t1.c2, u, m1);
  }
  fp6_add(s, f.c0, f.c1);
  l.c0 = L0.c0;
  fp2_add(l.c1, L0.c1, x);
  fp2_add(l.c2, L0.c2, y);
  fp6_mul(s, s, l);
  fp6_sub(s, s, t0);
  fp6_sub(f.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(f.c0, t0, t1);
  f_in = f;
}
// f = la * lb for two M-twist lines (the Miller loop's first step, where f = 1): the 6-product line product alone.
BLS_HD BLS_INLINE void fp12_line_pair(fp12& f, const fp2& ga0, const fp2& ga1, const fp2& ha1, const fp2& gb0,
                                      const fp2& gb1, const fp2& hb1) {
  fp2 p00, p11, phh, sa, sb, t;
  fp2_mul(p00, ga0, gb0);
  fp2_mul(p11, ga1, gb1);
  fp2_mul(phh, ha1, hb1);
  fp2_add_lazy(sa, ga0, ga1);
  fp2_add_lazy(sb, gb0, gb1);
  fp2_mul(t, sa, sb);
  fp2_sub(t, t, p00);
  fp2_sub(f.c0.c1, t, p11);
  fp2_mul_xi(t, phh);
  fp2_add(f.c0.c0, p00, t);
  f.c0.c2 = p11;
  fp2_set_zero(f.c1.c0);
  fp2_add_lazy(sa, ga0, ha1);
  fp2_add_lazy(sb, gb0, hb1);
  fp2_mul(t, sa, sb);
  fp2_sub(t, t, p00);
  fp2_sub(f.c1.c1, t, phh);
  fp2_add_lazy(sa, ga1, ha1);
  fp2_add_lazy(sb, gb1, hb1);
  fp2_mul(t, sa, sb);
  fp2_sub(t, t, p11);
  fp2_sub(f.c1.c2, t, phh);
}
BLS_HD BLS_MILLER_CALL void fp12_mul_line2(fp12& f_in, const fp2& ga0_in, const fp2& ga1_in, const fp2& ha1_in, const fp2& gb0_in,
                                    const fp2& gb1_in, const fp2& hb1_in) { fp12_mul_line2_inl(f_in, ga0_in, ga1_in, ha1_in, gb0_in, gb1_in, hb1_in); }
BLS_HD BLS_CALL void fp12_frobenius(fp12& r, const fp12& a_in, int j) {
  const fp12 a = a_in;
  // coefficient of w^k (k = 2i + h for a.c_h.c_i) is conj^j(c) * gamma_{j,k}
  const fp2* g = j == 1 ? FROB1 : (j == 2 ? FROB2 : FROB3);
  const fp2* src[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
  fp2* dst[6] = {&r.c0.c0, &r.c1.c0, &r.c0.c1, &r.c1.c1, &r.c0.c2, &r.c1.c2};
  fp2 tmp[6];
  for (int k = 0; k < 6; ++k) {
    fp2 c = *src[k];
    if (j & 1) fp2_conj(c, c);
    if (k == 0)
      tmp[k] = c;
    else
      fp2_mul(tmp[k], c, g[k]);
  }
  for (int k = 0; k < 6; ++k) *dst[k] = tmp[k];
}
// Body force-inlined into the exponentiation loop (pairing.h fp12_cyc_exp_xabs) so the Fp12 state stays in
// registers across the 63 squarings instead of round-tripping through the stack at every call.
BLS_HD BLS_INLINE void fp12_cyclotomic_sqr_body(fp12& r, const fp12& a) {
  // Granger-Scott: view a in Fp4^3 with Fp4 = Fp2[s]/(s^2 - xi), s = w^3... pairs
  // (g0,g1) := (c0.c0, c1.c1), (g2,g3) := (c1.c0, c0.c2), (g4,g5) := (c0.c1, c1.c2)
  fp2 z0 = a.c0.c0, z4 = a.c0.c1, z3 = a.c0.c2;
  fp2 z2 = a.c1.c0, z1 = a.c1.c1, z5 = a.c1.c2;
  fp2 t0, t1, t2, t3, tmp, tmp2;
  // fp4_sqr(z0, z1) -> (t0, t1)
  BLS_CYC_FP2_SQR(tmp, z0);
  BLS_CYC_FP2_SQR(tmp2, z1);
  fp2_mul_xi(t0, tmp2);
  fp2_add(t0, t0, tmp);
  fp2_add(t1, z0, z1);
  BLS_CYC_FP2_SQR(t1, t1);
  fp2_sub(t1, t1, tmp);
  fp2_sub(t1, t1, tmp2);
  // fp4_sqr(z2, z3) -> (t2, t3)
  BLS_CYC_FP2_SQR(tmp, z2);
  BLS_CYC_FP2_SQR(tmp2, z3);
  fp2_mul_xi(t2, tmp2);
  fp2_add(t2, t2, tmp);
  fp2_add(t3, z2, z3);
  BLS_CYC_FP2_SQR(t3, t3);
  fp2_sub(t3, t3, tmp);
  fp2_sub(t3, t3, tmp2);
  // fp4_sqr(z4, z5) -> (t4, t5)
  fp2 t4, t5;
  BLS_CYC_FP2_SQR(tmp, z4);
  BLS_CYC_FP2_SQR(tmp2, z5);
  fp2_mul_xi(t4, tmp2);
  fp2_add(t4, t4, tmp);
  fp2_add(t5, z4, z5);
  BLS_CYC_FP2_SQR(t5, t5);
  fp2_sub(t5, t5, tmp);
  fp2_sub(t5, t5, tmp2);
  // z0 = 3 t0 - 2 z0 ; z1 = 3 t1 + 2 z1
  fp2_sub(z0, t0, z0);
  fp2_dbl(z0, z0);
  fp2_add(z0, z0, t0);
  fp2_add(z1, t1, z1);
  fp2_dbl(z1, z1);
  fp2_add(z1, z1, t1);
  // z2 = 3 xi t5 + 2 z2 ; z3 = 3 t4 - 2 z3
  fp2_mul_xi(tmp, t5);
  fp2_add(z2, tmp, z2);
  fp2_dbl(z2, z2);
  fp2_add(z2, z2, tmp);
  fp2_sub(z3, t4, z3);
  fp2_dbl(z3, z3);
  fp2_add(z3, z3, t4);
  // z4 = 3 t2 - 2 z4 ; z5 = 3 t3 + 2 z5
  fp2_sub(z4, t2, z4);
  fp2_dbl(z4, z4);
  fp2_add(z4, z4, t2);
  fp2_add(z5, t3, z5);
  fp2_dbl(z5, z5);
  fp2_add(z5, z5, t3);
  r.c0.c0 = z0;
  r.c0.c1 = z4;
  r.c0.c2 = z3;
  r.c1.c0 = z2;
  r.c1.c1 = z1;
  r.c1.c2 = z5;
}

BLS_HD BLS_CALL void fp12_cyclotomic_sqr(fp12& r, const fp12& a_in) {
  const fp12 a = a_in;
  fp12 t;
  fp12_cyclotomic_sqr_body(t, a);
  r = t;
}

}  // namespace bls
