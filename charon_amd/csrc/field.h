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

// Test build (tests/test_operand_contract.py, host only): the device routines' operand contracts checked wherever the
// host runs the same per-lane code.  The product routines take operands below 2^382 (their carry elision, tools/
// gen_fp_asm.py _comba; every operand is canonical or a lazy sum below 2p), the Fp2 square and the modular add / sub
// canonical ones.  The host's lazy add / sub then stay unreduced as on the device, and a violation is counted.
#if defined(BLS_CONTRACT_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
namespace bls {
extern uint64_t g_contract_violations;
extern const char* g_contract_first;
extern uint64_t g_contract_lazy_operands;  // products that received an unreduced (lazy) operand: the check's coverage
}  // namespace bls
#define BLS_CONTRACT(cond, what)                                            \
  do {                                                                      \
    if (!(cond)) {                                                          \
      if (!::bls::g_contract_violations++) ::bls::g_contract_first = (what); \
    }                                                                       \
  } while (0)
#else
#define BLS_CONTRACT(cond, what) ((void)0)
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

#if defined(BLS_CONTRACT_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
static constexpr uint32_t P2_LIMBS_CONTRACT[12] = {0xffff5556u, 0x73fdffffu, 0x62a7ffffu, 0x3d57fffdu, 0xed61ec48u, 0xce61a541u, 0xe70a257eu, 0xc8ee9709u, 0x869759aeu, 0x96374f6cu, 0x72ffcd34u, 0x340223d4u};
// a < k p (k = 1, 2) by a borrow chain
inline bool fp_below_kp(const fp& a, int k) {
  int64_t br = 0;
  for (int i = 0; i < 12; ++i) {
    const uint64_t pk = k == 1 ? (uint64_t)P_LIMBS[i] : (uint64_t)P2_LIMBS_CONTRACT[i];
    br += (int64_t)a.v[i] - (int64_t)pk;
    br >>= 32;
  }
  return br < 0;
}
inline bool fp_canonical(const fp& a) { return fp_below_kp(a, 1); }
inline bool fp_product_operand(const fp& a) { return a.v[11] <= 0x3FFFFFFFu && fp_below_kp(a, 2); }
inline void fp_reduce_2p(fp& r, const fp& a) {  // a < 2p -> a mod p
  r = a;
  if (fp_canonical(a)) return;
  int64_t br = 0;
  for (int i = 0; i < 12; ++i) {
    br += (int64_t)a.v[i] - (int64_t)P_LIMBS[i];
    r.v[i] = (uint32_t)br;
    br >>= 32;
  }
}
#endif

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
  BLS_CONTRACT(fp_canonical(a) && fp_canonical(b), "fp_add: an operand is not canonical");
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
  BLS_CONTRACT(fp_canonical(a) && fp_canonical(b), "fp_sub: an operand is not canonical");
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
#if defined(BLS_CONTRACT_CHECK)
// the contract build: unreduced, as on the device (a + b, a + (p - b) for canonical a, b)
BLS_HD BLS_INLINE void fp_add_lazy(fp& r, const fp& a, const fp& b) {
  BLS_CONTRACT(fp_canonical(a) && fp_canonical(b), "fp_add_lazy: an operand is not canonical");
  uint64_t c = 0;
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
}
BLS_HD BLS_INLINE void fp_sub_lazy(fp& r, const fp& a, const fp& b) {
  BLS_CONTRACT(fp_canonical(a) && fp_canonical(b), "fp_sub_lazy: an operand is not canonical");
  int64_t c = 0;
  for (int i = 0; i < 12; ++i) {
    c += (int64_t)a.v[i] + (int64_t)P_LIMBS[i] - (int64_t)b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
}
#else
// host builds keep every value canonical
BLS_HD BLS_INLINE void fp_add_lazy(fp& r, const fp& a, const fp& b) { fp_add(r, a, b); }
BLS_HD BLS_INLINE void fp_sub_lazy(fp& r, const fp& a, const fp& b) { fp_sub(r, a, b); }
#endif
#endif

// r = a / 2 mod p (Montgomery form is preserved: (aR)/2 = (a/2)R): a + p when a is odd, then one right shift.
BLS_HD BLS_INLINE void fp_half(fp& r, const fp& a) {
  BLS_CONTRACT(fp_canonical(a), "fp_half: operand not canonical");
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
               "\n\ts_setpc_b64 s[30:31]\n"
               ".p2align 6\n.type bls_fp2_sqr_rt,@function\nbls_fp2_sqr_rt:\n\t" BLS_FP2_SQR_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n");
}
#ifndef BLS_LAZY_FP6
#define BLS_LAZY_FP6 0
#endif
#if BLS_LAZY_FP6 && !BLS_FP2_PAIR
// The lazy-reduction experiment's routines (tools/gen_fp_asm.py gen_fp2_mul2 / gen_fp2_mul3),
// generated on demand: `python3 charon_amd/tools/gen_fp_asm.py --lazy` writes the header below.
#include "../tools/fp_asm_lazy_gfx950.h"
__device__ __attribute__((used, noinline)) static void bls_fp2_lazy_routines() {
  asm volatile("s_endpgm\n.p2align 6\n.type bls_fp2_mul2_rt,@function\nbls_fp2_mul2_rt:\n\t" BLS_FP2_MUL2_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n"
               ".p2align 6\n.type bls_fp2_mul3_rt,@function\nbls_fp2_mul3_rt:\n\t" BLS_FP2_MUL3_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n");
}
#endif
#if BLS_FP2_PAIR
// The split-Fp2 build (verify_lat.hip): an Fp2 value is held in full on lanes l and l ^ 4, each computes one output
// coefficient of a product or square (tools/gen_fp_asm.py gen_fp2_mul_half / gen_fp2_sqr_half), then they swap.
__device__ __attribute__((used, noinline)) static void bls_fp2_half_routines() {
  asm volatile("s_endpgm\n.p2align 6\n.type bls_fp2_mul_half_rt,@function\nbls_fp2_mul_half_rt:\n\t"
               BLS_FP2_MUL_HALF_ASM_BODY "\n\ts_setpc_b64 s[30:31]\n"
               ".p2align 6\n.type bls_fp2_sqr_half_rt,@function\nbls_fp2_sqr_half_rt:\n\t" BLS_FP2_SQR_HALF_ASM_BODY
               "\n\ts_setpc_b64 s[30:31]\n");
}
// This lane's half: ~0 on lanes 4-7 of each group of eight (they form c1), 0 on lanes 0-3 (c0).
__device__ __forceinline__ uint32_t fp2p_mask() {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  return (lane & 4u) ? ~0u : 0u;
}
// The value of lane l ^ 4 (lanes 0-3 <-> 4-7 of each group of eight): row_shl:4 into banks 0 and 2 (lanes 0-3,
// 8-11 read 4-7, 12-15), row_shr:4 into banks 1 and 3.  All eight lanes must be active.
__device__ __forceinline__ uint32_t fp2p_xchg(uint32_t v) {
  const int a = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x104, 0xF, 0x5, false);
  return (uint32_t)__builtin_amdgcn_update_dpp(a, (int)v, 0x114, 0xF, 0xA, false);
}
__device__ __forceinline__ uint32_t fp2p_bfi(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b (v_bfi_b32, gcd30::bfi)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
#endif
// The routines read p from s16-s27 and -p^-1 mod 2^32 from s28 (tools/gen_fp_asm.py P_SGPR): the callers hold
// them there -- loaded from constant memory, uniform values the compiler keeps in those SGPRs across
// calls -- as inputs of every call, so the thirteen scalar moves leave the routines (each a full issue slot at one
// wave per SIMD, tools/isa_probe.hip).  The call's own address arithmetic then uses s[36:37].
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
static __constant__ uint32_t bls_p_sgpr[16] __attribute__((aligned(64))) = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau, 0xfffcfffdu, 0x00000000u, 0x00000000u, 0x00000000u};
// readfirstlane at each call: the values are uniform, and it keeps them scalar where the optimizer merged copies of
// them across divergent branches (a merged value is a VGPR, which an SGPR operand cannot take)
__device__ __forceinline__ uint32_t bls_p_word(int k) { return __builtin_amdgcn_readfirstlane(bls_p_sgpr[k]); }
__device__ __forceinline__ u32x8 bls_p_lo() {
  u32x8 v;
  v.s0 = bls_p_word(0); v.s1 = bls_p_word(1); v.s2 = bls_p_word(2); v.s3 = bls_p_word(3);
  v.s4 = bls_p_word(4); v.s5 = bls_p_word(5); v.s6 = bls_p_word(6); v.s7 = bls_p_word(7);
  return v;
}
__device__ __forceinline__ u32x4v bls_p_hi() {
  u32x4v v;
  v.s0 = bls_p_word(8); v.s1 = bls_p_word(9); v.s2 = bls_p_word(10); v.s3 = bls_p_word(11);
  return v;
}
#define BLS_P_SGPR_IN "{s[16:23]}"(bls_p_lo()), "{s[24:27]}"(bls_p_hi()), "{s28}"(bls_p_word(12))
#define BLS_ASM_CALL(fn)                                                                           \
  "s_getpc_b64 s[36:37]\n\ts_add_u32 s36, s36, " fn "@rel32@lo+4\n\ts_addc_u32 s37, s37, " fn \
  "@rel32@hi+12\n\ts_swappc_b64 s[30:31], s[36:37]\n\t"
#define BLS_CALL_CLOBBERS "s30", "s31", "s36", "s37", "scc"
__device__ __forceinline__ static u32x12 fp_mul_dev(u32x12 a, u32x12 b) {
  asm volatile(BLS_ASM_CALL("bls_fp_mul_rt") : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : BLS_P_SGPR_IN
               : BLS_FP_MUL_ASM_CLOBBERS, BLS_CALL_CLOBBERS);
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
#if defined(BLS_CONTRACT_CHECK)
  BLS_CONTRACT(fp_product_operand(a) && fp_product_operand(b), "fp_mul: an operand is not below 2p and 2^382");
  g_contract_lazy_operands += !fp_canonical(a) || !fp_canonical(b);
  fp_reduce_2p(a, a);
  fp_reduce_2p(b, b);
#endif
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
#if defined(BLS_CONTRACT_CHECK)
  BLS_CONTRACT(fp_product_operand(a), "fp_sqr: the operand is not below 2p and 2^382");
  fp_reduce_2p(a, a);
#endif
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
#ifndef BLS_POW_W
#define BLS_POW_W 5
#endif
#if BLS_FP2_PAIR && defined(__HIP_DEVICE_COMPILE__)
// The split-Fp2 build: right to left over the twin lanes.  Both lanes carry s = a^(2^i) and square it together while
// bit i is clear; at a set bit lane l (c0 side) squares while its twin l ^ 4 multiplies the accumulator by the same
// s, and one exchange gives the twin the new s.  One product of latency per exponent bit (top_bit + 1) instead of the
// window form's ~top_bit squarings + ~80 products on one lane, with the exchange only at set bits.  The accumulator
// lives on the c1 side and is exchanged once at the end.  All eight lanes of a group must be active (the twin
// products of this build require the same).
__device__ __forceinline__ void fp_pow_twin(fp& r, const fp& a, const uint32_t* e, int top_bit) {
  const uint32_t mul_lane = fp2p_mask();
  fp s = a, acc;
  bool started = false;
#pragma unroll 1
  for (int i = 0; i <= top_bit; ++i) {
#ifdef BLS_RACE_POLL
    if ((i & 63) == 63) BLS_RACE_POLL();
#endif
    const bool set = (e[i >> 5] >> (i & 31)) & 1u;  // wave-uniform
    if (set && started) {
      fp x, p, o;
#pragma unroll
      for (int k = 0; k < 12; ++k) x.v[k] = fp2p_bfi(mul_lane, acc.v[k], s.v[k]);
      fp_mul(p, x, s);  // c0 side: s^2 | c1 side: acc s
#pragma unroll
      for (int k = 0; k < 12; ++k) o.v[k] = fp2p_xchg(p.v[k]);
      acc = p;  // meaningful on the c1 side
#pragma unroll
      for (int k = 0; k < 12; ++k) s.v[k] = fp2p_bfi(mul_lane, o.v[k], p.v[k]);
    } else {
      if (set) {
        acc = s;
        started = true;
      }
      fp t;
      fp_mul(t, s, s);
      s = t;
    }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) r.v[k] = fp2p_bfi(mul_lane, acc.v[k], fp2p_xchg(acc.v[k]));
}
#endif
BLS_HD BLS_CALL void fp_pow(fp& r, const fp& a, const uint32_t* e, int top_bit) {
#if BLS_FP2_PAIR && defined(__HIP_DEVICE_COMPILE__)
  fp_pow_twin(r, a, e, top_bit);
  return;
#endif
  constexpr int W = BLS_POW_W;
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
      BLS_POW_CASE(6)
#if BLS_POW_W == 5
      BLS_POW_CASE(7) BLS_POW_CASE(8) BLS_POW_CASE(9) BLS_POW_CASE(10) BLS_POW_CASE(11)
      BLS_POW_CASE(12) BLS_POW_CASE(13) BLS_POW_CASE(14)
#endif
#undef BLS_POW_CASE
      default:
        w = tbl[(1 << (W - 1)) - 1];
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

// ---------------------------------------------------------------------------------- binary-GCD inversion
// Pornin's optimized binary GCD ("Optimized Binary GCD for Modular Inversion", 2020, Algorithm 2) with k = 31:
// 30 divsteps per outer iteration on 62-bit approximations (the low 30 bits and the top 32 bits of a and b at
// the longer one's length), then one signed 2x2 update of the full a, b (30-bit limbs) and of u, v mod p with an
// exact division by 2^30 (one Montgomery-style digit).  Invariant a = x u, b = x v (mod p); a reaches 0 and b = 1
// within len(a) + len(b) - 1 divsteps: 761 for a canonical input (< p, 381 bits), 763 for any input below 2^382
// (callers pass canonical values: fp_inv's operands are product or fp_add outputs, never fp_add_lazy sums).  ITERS =
// 27 runs 810 divsteps, covering both with a spare iteration; once a = 0 an iteration is a no-op (a stays 0).
// Every decision is a select on lane data: all lanes run the same instruction stream.  ~33k VALU per inversion
// against ~300k for the Fermat power x^(p-2) (455 products); inverse of 0 is 0, like the power.
// Result: x^-1 for the plain integer x = a_mont = aR, then one product by R^3 gives (aR)^-1 R^2 = a^-1 R.
namespace gcd30 {
static constexpr uint32_t M30 = 0x3fffffffu;
static constexpr uint32_t P30[13] = {0x3fffaaabu, 0x27fbffffu, 0x153ffffbu, 0x2affffacu, 0x30f6241eu,
                                     0x034a83dau, 0x112bf673u, 0x12e13ce1u, 0x2cd76477u, 0x1ed90d2eu,
                                     0x29a4b1bau, 0x3a8e5ff9u, 0x001a0111u};
static constexpr uint32_t PINV30 = 0x3ffcfffdu;  // -p^-1 mod 2^30
static constexpr int ITERS = 27;

// Lane masks as VGPR values and selects by v_bfi_b32.  Written as (non-volatile) asm on the device so the compiler
// cannot turn "x & mask" back into a v_cndmask_b32_e32 on VCC, which issues at ~19 cycles on gfx950 against ~4.4
// for v_bfi_b32 (profiles/r02_sel_probe.txt).
#if defined(__HIP_DEVICE_COMPILE__)
BLS_HD BLS_INLINE uint32_t mask_bit0(uint32_t x) {  // all ones if x is odd
  uint32_t m;
  asm("v_bfe_i32 %0, %1, 0, 1" : "=v"(m) : "v"(x));
  return m;
}
BLS_HD BLS_INLINE uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, bitwise
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
#else
BLS_HD BLS_INLINE uint32_t mask_bit0(uint32_t x) { return 0u - (x & 1u); }
BLS_HD BLS_INLINE uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
#endif
BLS_HD BLS_INLINE uint32_t mask_eq(uint32_t a, uint32_t b) {  // all ones if a == b (a ^ b < 2^31)
  return (uint32_t)((int32_t)((a ^ b) - 1u) >> 31);
}

// One divstep on the 62-bit approximations a = (ah:al), b = (bh:bl) and the transition factors:
//   a odd:  d = a - b;  b <- min(a, b);  a <- |d| / 2;  (f0, f1) <- (+-(f0 - f1), 2 (a < b ? f0 : f1))
//   a even: a <- a / 2;  f1 <- 2 f1          (likewise g)
// i.e. Pornin's "if a odd: if a < b: swap; a -= b" followed by the halving, without a branch or a VCC select.
#if defined(__HIP_DEVICE_COMPILE__)
BLS_HD BLS_INLINE void divstep(uint32_t& al, uint32_t& ah, uint32_t& bl, uint32_t& bh, uint32_t& f0, uint32_t& g0,
                               uint32_t& f1, uint32_t& g1) {
  uint32_t om, s, sw, dl, dh, t;
  asm("v_bfe_i32 %[om], %[al], 0, 1\n\t"
      "v_sub_co_u32_e32 %[dl], vcc, %[al], %[bl]\n\t"
      "v_subb_co_u32_e32 %[dh], vcc, %[ah], %[bh], vcc\n\t"
      "v_ashrrev_i32_e32 %[s], 31, %[dh]\n\t"
      "v_and_b32_e32 %[sw], %[om], %[s]\n\t"
      "v_xor_b32_e32 %[dl], %[dl], %[s]\n\t"
      "v_xor_b32_e32 %[dh], %[dh], %[s]\n\t"
      "v_sub_co_u32_e32 %[dl], vcc, %[dl], %[s]\n\t"
      "v_subb_co_u32_e32 %[dh], vcc, %[dh], %[s], vcc\n\t"
      "v_bfi_b32 %[bl], %[sw], %[al], %[bl]\n\t"
      "v_bfi_b32 %[bh], %[sw], %[ah], %[bh]\n\t"
      "v_bfi_b32 %[al], %[om], %[dl], %[al]\n\t"
      "v_bfi_b32 %[ah], %[om], %[dh], %[ah]\n\t"
      "v_alignbit_b32 %[al], %[ah], %[al], 1\n\t"
      "v_lshrrev_b32_e32 %[ah], 1, %[ah]\n\t"
      "v_sub_u32_e32 %[t], %[f0], %[f1]\n\t"
      "v_xor_b32_e32 %[t], %[t], %[sw]\n\t"
      "v_sub_u32_e32 %[t], %[t], %[sw]\n\t"
      "v_bfi_b32 %[f1], %[sw], %[f0], %[f1]\n\t"
      "v_lshlrev_b32_e32 %[f1], 1, %[f1]\n\t"
      "v_bfi_b32 %[f0], %[om], %[t], %[f0]\n\t"
      "v_sub_u32_e32 %[t], %[g0], %[g1]\n\t"
      "v_xor_b32_e32 %[t], %[t], %[sw]\n\t"
      "v_sub_u32_e32 %[t], %[t], %[sw]\n\t"
      "v_bfi_b32 %[g1], %[sw], %[g0], %[g1]\n\t"
      "v_lshlrev_b32_e32 %[g1], 1, %[g1]\n\t"
      "v_bfi_b32 %[g0], %[om], %[t], %[g0]"
      : [al] "+v"(al), [ah] "+v"(ah), [bl] "+v"(bl), [bh] "+v"(bh), [f0] "+v"(f0), [g0] "+v"(g0), [f1] "+v"(f1),
        [g1] "+v"(g1), [om] "=&v"(om), [s] "=&v"(s), [sw] "=&v"(sw), [dl] "=&v"(dl), [dh] "=&v"(dh), [t] "=&v"(t)
      :
      : "vcc");
}
#else
BLS_HD BLS_INLINE void divstep(uint32_t& al, uint32_t& ah, uint32_t& bl, uint32_t& bh, uint32_t& f0, uint32_t& g0,
                               uint32_t& f1, uint32_t& g1) {
  const uint64_t a = (uint64_t)ah << 32 | al, b = (uint64_t)bh << 32 | bl;
  const uint32_t om = mask_bit0(al);
  const int64_t d = (int64_t)(a - b);
  const uint32_t s = (uint32_t)(d >> 63), sw = om & s;
  const uint64_t ad = d < 0 ? (uint64_t)-d : (uint64_t)d;
  const uint64_t nb = sw ? a : b, na = (om ? ad : a) >> 1;
  const uint32_t tf = ((f0 - f1) ^ sw) - sw, tg = ((g0 - g1) ^ sw) - sw;
  f1 = bfi(sw, f0, f1) << 1;
  g1 = bfi(sw, g0, g1) << 1;
  f0 = bfi(om, tf, f0);
  g0 = bfi(om, tg, g0);
  al = (uint32_t)na;
  ah = (uint32_t)(na >> 32);
  bl = (uint32_t)nb;
  bh = (uint32_t)(nb >> 32);
}
#endif

// limbs: 12 x 32 -> 13 x 30
BLS_HD BLS_INLINE void to30(int32_t* o, const uint32_t* x) {
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int b = 30 * i, w = b >> 5, s = b & 31;
    uint64_t v = x[w];
    if (w + 1 < 12) v |= (uint64_t)x[w + 1] << 32;
    o[i] = (int32_t)((uint32_t)(v >> s) & M30);
  }
}
// 13 x 30 (non-negative, each < 2^30, value < 2^384) -> 12 x 32
BLS_HD BLS_INLINE void from30(uint32_t* o, const int32_t* x) {
#pragma unroll
  for (int w = 0; w < 12; ++w) {
    const int b = 32 * w, i = b / 30, s = b % 30;
    uint64_t v = (uint64_t)(uint32_t)x[i] >> s;
    v |= (uint64_t)(uint32_t)x[i + 1] << (30 - s);
    if (i + 2 < 13 && 60 - s < 32) v |= (uint64_t)(uint32_t)x[i + 2] << (60 - s);
    o[w] = (uint32_t)v;
  }
}
// r = (x f + y g) / 2^30 for 30-bit limb vectors (top limb signed); the low 30 bits of x f + y g are zero.
BLS_HD BLS_INLINE void lin_shift(int32_t* r, const int32_t* x, const int32_t* y, int32_t f, int32_t g) {
  int64_t c = (int64_t)x[0] * f + (int64_t)y[0] * g;
  c >>= 30;
#pragma unroll
  for (int i = 1; i < 13; ++i) {
    c += (int64_t)x[i] * f + (int64_t)y[i] * g;
    r[i - 1] = (int32_t)((uint32_t)c & M30);
    c >>= 30;
  }
  r[12] = (int32_t)c;
}
// r = |r| (top limb signed), returns the mask -1 if r was negative
BLS_HD BLS_INLINE int32_t cond_neg(int32_t* r) {
  const int32_t s = r[12] >> 31;
  int32_t c = s & 1;  // -r = (r ^ -1) + 1 limb-wise
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int32_t t = (r[i] ^ (s & (int32_t)M30)) + c;
    r[i] = t & (int32_t)M30;
    c = t >> 30;
  }
  r[12] = (r[12] ^ s) + c;
  return s;
}
// r = (u f + v g) / 2^30 mod p, for u, v in [0, p); result in [0, p)
BLS_HD BLS_INLINE void lin_mod(int32_t* r, const int32_t* u, const int32_t* v, int32_t f, int32_t g) {
  int64_t c = (int64_t)u[0] * f + (int64_t)v[0] * g;
  const int32_t k = (int32_t)(((uint32_t)c * PINV30) & M30);
  c += (int64_t)k * (int32_t)P30[0];
  c >>= 30;
#pragma unroll
  for (int i = 1; i < 13; ++i) {
    c += (int64_t)u[i] * f + (int64_t)v[i] * g + (int64_t)k * (int32_t)P30[i];
    r[i - 1] = (int32_t)((uint32_t)c & M30);
    c >>= 30;
  }
  r[12] = (int32_t)c;  // r in (-p, 2p)
  // r < 0: r += p
  int32_t s = r[12] >> 31;
  int32_t cc = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int32_t t = r[i] + ((int32_t)P30[i] & s) + cc;
    r[i] = i < 12 ? (t & (int32_t)M30) : t;
    cc = t >> 30;
  }
  // r >= p: r -= p
  int32_t d[13];
  cc = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int32_t t = r[i] - (int32_t)P30[i] + cc;
    d[i] = i < 12 ? (t & (int32_t)M30) : t;
    cc = t >> 30;
  }
  s = d[12] >> 31;  // borrow: keep r
#pragma unroll
  for (int i = 0; i < 13; ++i) r[i] = (int32_t)bfi((uint32_t)s, (uint32_t)r[i], (uint32_t)d[i]);
}
}  // namespace gcd30

BLS_HD BLS_CALL void fp_inv(fp& r, const fp& a_in) {
  using namespace gcd30;
  int32_t a[13], b[13], u[13], v[13];
  to30(a, a_in.v);
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    b[i] = (int32_t)P30[i];
    u[i] = i == 0;
    v[i] = 0;
  }
  for (int it = 0; it < ITERS; ++it) {
    // n = max(len(a), len(b), 62): bits [n-32, n) of a and b, and their low 30 bits
    uint32_t top = 0;
    int hi = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const uint32_t t = (uint32_t)(a[i] | b[i]);
      hi = t ? i : hi;
      top = t ? t : top;
    }
    int n = 30 * hi + (32 - __builtin_clz(top | 1u));
    n = n < 62 ? 62 : n;
    const int pos = n - 32, L = (pos * 2185) >> 16, sh = pos - 30 * L;
    uint32_t wa0 = 0, wa1 = 0, wb0 = 0, wb1 = 0;  // 64-bit windows of a and b starting at limb L
#pragma unroll
    for (int i = 0; i < 12; ++i) {  // a, b <= p < 2^381: the window starts in limb 11 at most
      const uint32_t m = mask_eq((uint32_t)i, (uint32_t)L);
      uint64_t xa = (uint64_t)(uint32_t)a[i] | ((uint64_t)(uint32_t)a[i + 1] << 30);
      uint64_t xb = (uint64_t)(uint32_t)b[i] | ((uint64_t)(uint32_t)b[i + 1] << 30);
      if (i + 2 < 13) {
        xa |= (uint64_t)(uint32_t)a[i + 2] << 60;
        xb |= (uint64_t)(uint32_t)b[i + 2] << 60;
      }
      wa0 = bfi(m, (uint32_t)xa, wa0);
      wa1 = bfi(m, (uint32_t)(xa >> 32), wa1);
      wb0 = bfi(m, (uint32_t)xb, wb0);
      wb1 = bfi(m, (uint32_t)(xb >> 32), wb1);
    }
    const uint64_t wa = (uint64_t)wa1 << 32 | wa0, wb = (uint64_t)wb1 << 32 | wb0;
    const uint64_t ab = (uint64_t)(uint32_t)(wa >> sh) << 30 | (uint32_t)a[0];
    const uint64_t bb = (uint64_t)(uint32_t)(wb >> sh) << 30 | (uint32_t)b[0];
    uint32_t al = (uint32_t)ab, ah = (uint32_t)(ab >> 32), bl = (uint32_t)bb, bh = (uint32_t)(bb >> 32);
    uint32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 5
    for (int j = 0; j < 30; ++j) divstep(al, ah, bl, bh, f0, g0, f1, g1);
    int32_t na[13], nb[13];
    lin_shift(na, a, b, f0, g0);
    lin_shift(nb, a, b, f1, g1);
    const int32_t sa = cond_neg(na), sb = cond_neg(nb);
    f0 = (f0 ^ sa) - sa;
    g0 = (g0 ^ sa) - sa;
    f1 = (f1 ^ sb) - sb;
    g1 = (g1 ^ sb) - sb;
    int32_t nu[13], nv[13];
    lin_mod(nu, u, v, f0, g0);
    lin_mod(nv, u, v, f1, g1);
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      a[i] = na[i];
      b[i] = nb[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  fp y, r3;
  from30(y.v, v);
#pragma unroll
  for (int i = 0; i < 12; ++i) r3.v[i] = R3_LIMBS[i];
  fp_mul(r, y, r3);
}

// Fermat inverse (kept for the host tests that cross-check the binary GCD)
BLS_HD BLS_INLINE void fp_inv_pow(fp& r, const fp& a) { fp_pow(r, a, EXP_P_MINUS_2, 380); }

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
