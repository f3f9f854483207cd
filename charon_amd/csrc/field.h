// Fp arithmetic for BLS12-381 on gfx950: 381-bit prime field, 12 x 32-bit limbs per element,
// Montgomery form with R = 2^384.  One lane owns one element; every carry chain stays in VGPRs
// (32x32->64 v_mad_u64_u32 + v_add_co/v_addc_co).  All values are kept fully reduced in [0, p),
// so equality and zero tests are limb compares.
//
// This replaces the mcl Fp layer that herumi/bls-eth-go-binary v1.32.1 links into charon's
// tbls.Herumi (/root/reference/tbls/herumi.go:12); see DESIGN.md for the roofline unit
// (one fp_mul = one "Fp-mul-equivalent").
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BLS_HD __host__ __device__
#define BLS_INLINE static __forceinline__
#else
#define BLS_HD
#define BLS_INLINE static inline
#endif
#define BLS_NOINLINE static __attribute__((noinline))
// Mid-level building blocks (Fp6/Fp12 products, curve steps, hash stages) are real calls: their
// bodies are emitted once, so a kernel's instruction footprint stays within the instruction cache
// and compile time stays linear.  Fp and Fp2 arithmetic is inlined into them.
#ifndef BLS_CALL
#define BLS_CALL static __attribute__((noinline))
#endif

namespace bls {

struct fp {
  uint32_t v[12];
};
struct fp2 {
  fp c0, c1;
};

}  // namespace bls

#include "bls_constants.h"

#if defined(BLS_COUNT_OPS)
namespace bls {
// Host-only instrumentation (tests/native builds): counts the Fp multiplications an operation
// performs -- the algorithmic unit behind bench.py's roofline.
extern thread_local uint64_t g_fp_mul_count;
extern thread_local uint64_t g_fp_sqr_count;
}  // namespace bls
#define BLS_COUNT_MUL() (++::bls::g_fp_mul_count)
#define BLS_COUNT_SQR() (++::bls::g_fp_sqr_count)
#else
#define BLS_COUNT_MUL() ((void)0)
#define BLS_COUNT_SQR() ((void)0)
#endif

namespace bls {

BLS_HD BLS_INLINE void fp_set_zero(fp& r) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = 0;
}

BLS_HD BLS_INLINE void fp_set_one(fp& r) { r = FP_ONE; }

BLS_HD BLS_INLINE bool fp_is_zero(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i];
  return acc == 0;
}

BLS_HD BLS_INLINE bool fp_eq(const fp& a, const fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

#if defined(__HIP_DEVICE_COMPILE__)
}  // namespace bls
#include "fp_asm_gfx950.h"
namespace bls {
// Device: each modular add / sub / negation is ONE asm block (tools/gen_fp_asm.py gen_add / gen_sub): a single
// VCC carry chain, the borrow turned into a VGPR lane mask, and v_bfi_b32 / v_and_b32 selects -- 37 VALU, no
// s_nop padding (compiled C++ interleaves two carry chains on VCC and an SGPR pair and pays an s_nop per step)
// and no VOP2 v_cndmask_b32_e32 (~19 cycles on gfx950).  Measured: profiles/r02_op_probe.txt.
#define BLS_FP12_OUT(x) "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), \
                        "=&v"(x[7]), "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11])
#define BLS_FP12_IN(x) "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]), \
                       "v"(x[8]), "v"(x[9]), "v"(x[10]), "v"(x[11])
// r = a + b mod p
BLS_HD BLS_INLINE void fp_add(fp& r, const fp& a, const fp& b) {
  uint32_t o[12], t[12], m;
  asm volatile(BLS_FP_ADD_ASM : BLS_FP12_OUT(o), BLS_FP12_OUT(t), "=&v"(m)
               : BLS_FP12_IN(a.v), BLS_FP12_IN(b.v), BLS_FP12_IN(P_LIMBS) : "vcc");
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = o[i];
}
// r = a - b mod p
BLS_HD BLS_INLINE void fp_sub(fp& r, const fp& a, const fp& b) {
  uint32_t o[12], t[12], m;
  asm volatile(BLS_FP_SUB_ASM : BLS_FP12_OUT(o), BLS_FP12_OUT(t), "=&v"(m)
               : BLS_FP12_IN(a.v), BLS_FP12_IN(b.v), BLS_FP12_IN(P_LIMBS) : "vcc");
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = o[i];
}
#else
// r = a + b mod p
BLS_HD BLS_INLINE void fp_add(fp& r, const fp& a, const fp& b) {
  uint32_t s[12];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    s[i] = (uint32_t)c;
    c >>= 32;
  }
  // s < 2p < 2^384, no carry out; subtract p and keep if no borrow
  uint32_t d[12];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)s[i] - P_LIMBS[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const bool keep_s = br < 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = keep_s ? s[i] : d[i];
}

// r = a - b mod p
BLS_HD BLS_INLINE void fp_sub(fp& r, const fp& a, const fp& b) {
  uint32_t d[12];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)a.v[i] - b.v[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const uint32_t mask = br < 0 ? 0xffffffffu : 0u;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)d[i] + (P_LIMBS[i] & mask);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
}

#endif

#if defined(__HIP_DEVICE_COMPILE__)
// Product operands only (see gen_fp_asm.py gen_add_lazy / gen_sub_lazy): a + b and a + (p - b) left unreduced in
// [0, 2p).  The Montgomery product reduces any operands with a*b < p*2^384 to a canonical result.
BLS_HD BLS_INLINE void fp_add_lazy(fp& r, const fp& a, const fp& b) {
  uint32_t o[12];
  asm volatile(BLS_FP_ADD_LAZY_ASM : BLS_FP12_OUT(o) : BLS_FP12_IN(a.v), BLS_FP12_IN(b.v) : "vcc");
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = o[i];
}
BLS_HD BLS_INLINE void fp_sub_lazy(fp& r, const fp& a, const fp& b) {
  uint32_t o[12], t[12];
  asm volatile(BLS_FP_SUB_LAZY_ASM : BLS_FP12_OUT(o), BLS_FP12_OUT(t)
               : BLS_FP12_IN(a.v), BLS_FP12_IN(b.v), BLS_FP12_IN(P_LIMBS) : "vcc");
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = o[i];
}
BLS_HD BLS_INLINE void fp_neg(fp& r, const fp& a) {
  uint32_t o[12], t[12], m;
  asm volatile(BLS_FP_NEG_ASM : BLS_FP12_OUT(o), BLS_FP12_OUT(t), "=&v"(m) : BLS_FP12_IN(a.v), BLS_FP12_IN(P_LIMBS)
               : "vcc");
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = o[i];
}
#else
BLS_HD BLS_INLINE void fp_neg(fp& r, const fp& a) {
  fp z;
  fp_set_zero(z);
  fp_sub(r, z, a);
}
// host builds keep every value canonical
BLS_HD BLS_INLINE void fp_add_lazy(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
BLS_HD BLS_INLINE void fp_sub_lazy(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
#endif

// r = a / 2 mod p (Montgomery form is preserved: (aR)/2 = (a/2)R): a + p when a is odd, then one right shift.
BLS_HD BLS_INLINE void fp_half(fp& r, const fp& a) {
  const uint32_t m = 0u - (a.v[0] & 1u);
  uint32_t t[12];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)a.v[i] + (P_LIMBS[i] & m);
    t[i] = (uint32_t)c;
    c >>= 32;
  }
#pragma unroll
  for (int i = 0; i < 11; ++i) r.v[i] = (t[i] >> 1) | (t[i + 1] << 31);
  r.v[11] = t[11] >> 1;
}

BLS_HD BLS_INLINE void fp_dbl(fp& r, const fp& a) { fp_add(r, a, a); }

// Montgomery product r = a*b*R^-1 mod p.  CIOS with the "no-carry" shortcut: p's top limb
// 0x1a0111ea < 2^31 - 1, so the running sum never needs a 14th word.
BLS_HD BLS_INLINE void fp_mul_impl(fp& r, const fp& a, const fp& b) {
  uint32_t t[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t A = (uint64_t)a.v[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * P_INV32;
    uint64_t C = (uint64_t)m * P_LIMBS[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; ++j) {
      A = (uint64_t)a.v[j] * bi + t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * P_LIMBS[j] + t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  // t < 2p: conditional subtraction
  uint32_t d[12];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)t[i] - P_LIMBS[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const bool keep_t = br < 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = keep_t ? t[i] : d[i];
}

// gfx950: the product is one hand-scheduled routine (tools/gen_fp_asm.py) emitted ONCE into the
// code object and reached by an s_swappc from inline asm.  Because the compiler sees an asm block
// rather than a call, the only registers it must treat as clobbered are the ones the routine really
// touches (v24-v39, s16-s31, vcc) -- not the ABI's whole caller-saved set -- so values live across
// a product stay in registers instead of being saved to scratch around every multiplication.
// Operands are pinned: a in v[0:11] (result out), b in v[12:23].
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t u32x12 __attribute__((ext_vector_type(12)));
// Never called: hosts the routine's code (entered only at the local label).
__device__ __attribute__((used, noinline)) static void bls_fp_asm_routines() {
  asm volatile("s_endpgm\n.p2align 6\n.type bls_fp_mul_rt,@function\nbls_fp_mul_rt:\n\t" BLS_FP_MUL_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n"
               ".p2align 6\n.type bls_fp2_mul_rt,@function\nbls_fp2_mul_rt:\n\t" BLS_FP2_MUL_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n");
}
#define BLS_ASM_CALL(fn)                                                                           \
  "s_getpc_b64 s[16:17]\n\ts_add_u32 s16, s16, " fn "@rel32@lo+4\n\ts_addc_u32 s17, s17, " fn \
  "@rel32@hi+12\n\ts_swappc_b64 s[30:31], s[16:17]\n\t"
__device__ __forceinline__ static u32x12 fp_mul_dev(u32x12 a, u32x12 b) {
  asm volatile(BLS_ASM_CALL("bls_fp_mul_rt") : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : BLS_FP_MUL_ASM_CLOBBERS,
               "s30", "s31", "scc");
  return a;
}
BLS_HD BLS_INLINE u32x12 fp_to_vec(const fp& a) {
  u32x12 v;
  v.s0 = a.v[0]; v.s1 = a.v[1]; v.s2 = a.v[2]; v.s3 = a.v[3]; v.s4 = a.v[4]; v.s5 = a.v[5];
  v.s6 = a.v[6]; v.s7 = a.v[7]; v.s8 = a.v[8]; v.s9 = a.v[9]; v.sA = a.v[10]; v.sB = a.v[11];
  return v;
}
BLS_HD BLS_INLINE void fp_from_vec(fp& r, const u32x12& v) {
  r.v[0] = v.s0; r.v[1] = v.s1; r.v[2] = v.s2; r.v[3] = v.s3; r.v[4] = v.s4; r.v[5] = v.s5;
  r.v[6] = v.s6; r.v[7] = v.s7; r.v[8] = v.s8; r.v[9] = v.s9; r.v[10] = v.sA; r.v[11] = v.sB;
}
BLS_HD BLS_INLINE void fp_mul(fp& r, const fp& a, const fp& b) { fp_from_vec(r, fp_mul_dev(fp_to_vec(a), fp_to_vec(b))); }
BLS_HD BLS_INLINE void fp_sqr(fp& r, const fp& a) {
  const u32x12 v = fp_to_vec(a);
  fp_from_vec(r, fp_mul_dev(v, v));
}
#else
#if defined(BLS_HOST_FAST_MUL)
// Host CPU baseline build (tests/native/cpu_baseline.cpp): the same Montgomery product (R = 2^384) on 6 x 64-bit
// limbs with 64x64->128 multiplies -- x86-64's native width -- instead of the 12 x 32-bit form the GPU uses.
// Little-endian: the 12 32-bit limbs ARE the 6 64-bit limbs.  p's top limb < 2^63: no-carry CIOS.
static inline void fp_mul_impl64(fp& r, const fp& a, const fp& b) {
  typedef unsigned __int128 u128;
  static const uint64_t P64[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                  0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
  const uint64_t PINV64 = 0x89f3fffcfffcfffdull;
  uint64_t A[6], B[6], t[6] = {0, 0, 0, 0, 0, 0};
  __builtin_memcpy(A, a.v, 48);
  __builtin_memcpy(B, b.v, 48);
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)A[0] * B[i] + t[0];
    t[0] = (uint64_t)x;
    const uint64_t m = t[0] * PINV64;
    u128 y = (u128)m * P64[0] + t[0];
    for (int j = 1; j < 6; ++j) {
      x = (u128)A[j] * B[i] + t[j] + (uint64_t)(x >> 64);
      t[j] = (uint64_t)x;
      y = (u128)m * P64[j] + t[j] + (uint64_t)(y >> 64);
      t[j - 1] = (uint64_t)y;
    }
    t[5] = (uint64_t)(y >> 64) + (uint64_t)(x >> 64);
  }
  uint64_t d[6];
  unsigned char br = 0;
  for (int i = 0; i < 6; ++i) {
    const u128 s = (u128)t[i] - P64[i] - br;
    d[i] = (uint64_t)s;
    br = (unsigned char)((s >> 64) != 0);
  }
  __builtin_memcpy(r.v, br ? t : d, 48);
}
#endif
BLS_HD BLS_NOINLINE fp fp_mul_v(fp a, fp b) {
  BLS_COUNT_MUL();
  fp r;
#if defined(BLS_HOST_FAST_MUL)
  fp_mul_impl64(r, a, b);
#else
  fp_mul_impl(r, a, b);
#endif
  return r;
}
BLS_HD BLS_NOINLINE fp fp_sqr_v(fp a) {
  BLS_COUNT_SQR();
  fp r;
#if defined(BLS_HOST_FAST_MUL)
  fp_mul_impl64(r, a, a);
#else
  fp_mul_impl(r, a, a);
#endif
  return r;
}
BLS_HD BLS_INLINE void fp_mul(fp& r, const fp& a, const fp& b) { r = fp_mul_v(a, b); }
BLS_HD BLS_INLINE void fp_sqr(fp& r, const fp& a) { r = fp_sqr_v(a); }
#endif

// r = a^e for a fixed exponent given as little-endian 32-bit limbs whose top set bit is top_bit.
// Left-to-right sliding window of 5 bits over the odd powers a, a^3, .., a^31: for the ~380-bit
// exponents used here (p-2, (p+1)/4, (p-3)/4, Hamming weight ~229) that is ~380 squarings + ~80
// products instead of ~380 + 229.  The exponent is the same for every lane, so every branch and
// table index is wave-uniform.
BLS_HD BLS_CALL void fp_pow(fp& r, const fp& a, const uint32_t* e, int top_bit) {
  constexpr int W = 5;
  fp tbl[1 << (W - 1)];
  fp a2;
  tbl[0] = a;
  fp_sqr(a2, a);
  for (int k = 1; k < (1 << (W - 1)); ++k) fp_mul(tbl[k], tbl[k - 1], a2);
  auto bit = [&](int i) { return (e[i >> 5] >> (i & 31)) & 1u; };
  fp acc;
  bool started = false;
  int i = top_bit;
  while (i >= 0) {
    if (!bit(i)) {
      if (started) fp_sqr(acc, acc);
      --i;
      continue;
    }
    int j = i - (W - 1) < 0 ? 0 : i - (W - 1);
    while (!bit(j)) ++j;  // window [i..j] ends on a set bit, so its value is odd
    uint32_t v = 0;
    for (int k = i; k >= j; --k) {
      v = (v << 1) | bit(k);
      if (started) fp_sqr(acc, acc);
    }
    // the table index is wave-uniform: select through a switch of constant indices so the table stays in
    // registers (a dynamic index would put it in scratch and cost a memory round trip per window)
    fp w;
    switch (v >> 1) {
#define BLS_POW_CASE(k) \
  case k:               \
    w = tbl[k];         \
    break;
      BLS_POW_CASE(0) BLS_POW_CASE(1) BLS_POW_CASE(2) BLS_POW_CASE(3) BLS_POW_CASE(4) BLS_POW_CASE(5)
      BLS_POW_CASE(6) BLS_POW_CASE(7) BLS_POW_CASE(8) BLS_POW_CASE(9) BLS_POW_CASE(10) BLS_POW_CASE(11)
      BLS_POW_CASE(12) BLS_POW_CASE(13) BLS_POW_CASE(14)
#undef BLS_POW_CASE
      default:
        w = tbl[15];
        break;
    }
    if (started) {
      fp_mul(acc, acc, w);
    } else {
      acc = w;
      started = true;
    }
    i = j - 1;
  }
  r = acc;
}

BLS_HD BLS_INLINE void fp_mul_small(fp& r, const fp& a, uint32_t k) {
  // r = k*a mod p for tiny k by repeated doubling/adding (k <= 16)
  fp acc;
  fp_set_zero(acc);
  fp base = a;
  while (k) {
    if (k & 1) fp_add(acc, acc, base);
    fp_add(base, base, base);
    k >>= 1;
  }
  r = acc;
}

BLS_HD BLS_INLINE void fp_inv(fp& r, const fp& a) { fp_pow(r, a, EXP_P_MINUS_2, 380); }

// Returns true and r = sqrt(a) when a is a square (p = 3 mod 4: r = a^((p+1)/4)).
BLS_HD BLS_INLINE bool fp_sqrt(fp& r, const fp& a) {
  fp s, s2;
  fp_pow(s, a, EXP_SQRT, 378);
  fp_sqr(s2, s);
  r = s;
  return fp_eq(s2, a);
}

BLS_HD BLS_INLINE void fp_to_mont(fp& r, const fp& a) {
  fp r2;
#pragma unroll
  for (int i = 0; i < 12; ++i) r2.v[i] = R2_LIMBS[i];
  fp_mul(r, a, r2);
}

BLS_HD BLS_INLINE void fp_from_mont(fp& r, const fp& a) {
  fp one;
#pragma unroll
  for (int i = 0; i < 12; ++i) one.v[i] = i == 0 ? 1u : 0u;
  fp_mul(r, a, one);
}

// Plain (non-Montgomery) value compare: is a > (p-1)/2 ?  'a' must be canonical (from_mont'd).
BLS_HD BLS_INLINE bool fp_plain_gt_half(const fp& a) {
  // (p-1)/2 limbs
  constexpr uint32_t H[12] = {0xffffd555u, 0xdcff7fffu, 0x58a9ffffu, 0x0f55ffffu, 0x7b587b12u, 0xb3986950u,
                              0x79c2895fu, 0xb23ba5c2u, 0x21a5d66bu, 0x258dd3dbu, 0x1cbff34du, 0x0d0088f5u};
  // compute H - a; borrow => a > H
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)H[i] - a.v[i];
    br >>= 32;
  }
  return br < 0;
}

// Is the plain value a < p ?
BLS_HD BLS_INLINE bool fp_plain_lt_p(const fp& a) {
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)a.v[i] - P_LIMBS[i];
    br >>= 32;
  }
  return br < 0;
}

// 48 big-endian bytes -> plain limbs
BLS_HD BLS_INLINE void fp_plain_from_be48(fp& r, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint8_t* q = b + 44 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}

BLS_HD BLS_INLINE void fp_plain_to_be48(uint8_t* b, const fp& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.v[i] >> 24);
    q[1] = (uint8_t)(a.v[i] >> 16);
    q[2] = (uint8_t)(a.v[i] >> 8);
    q[3] = (uint8_t)a.v[i];
  }
}

}  // namespace bls
