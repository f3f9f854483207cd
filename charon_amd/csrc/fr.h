// Scalar field Fr (r = 0x73ed...0001, 255 bits): 8 x 32-bit limbs, Montgomery form R = 2^256.
// Used for the Lagrange coefficients of ThresholdAggregate (herumi Sign.Recover,
// /root/reference/tbls/herumi.go:276) -- lambda_i = prod_{j!=i} x_j / (x_j - x_i) at x = 0.
#pragma once
#include "field.h"

namespace bls {

struct fr {
  uint32_t v[8];
};

BLS_HD BLS_INLINE void fr_add(fr& r, const fr& a, const fr& b) {
  uint32_t s[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    s[i] = (uint32_t)c;
    c >>= 32;
  }
  uint32_t d[8];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    br += (int64_t)s[i] - FR_LIMBS[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const bool keep_s = (br < 0) && (c == 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = keep_s ? s[i] : d[i];
}

BLS_HD BLS_INLINE void fr_sub(fr& r, const fr& a, const fr& b) {
  uint32_t d[8];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    br += (int64_t)a.v[i] - b.v[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const uint32_t mask = br < 0 ? 0xffffffffu : 0u;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)d[i] + (FR_LIMBS[i] & mask);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
}

// CIOS Montgomery product (r's top limb 0x73eda753 < 2^31 - 1: no-carry variant applies)

BLS_HD BLS_CALL void fr_mul(fr& r, const fr& a, const fr& b) {
  uint32_t t[8];
  for (int i = 0; i < 8; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t A = (uint64_t)a.v[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * FR_INV32;
    uint64_t C = (uint64_t)m * FR_LIMBS[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      A = (uint64_t)a.v[j] * bi + t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * FR_LIMBS[j] + t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[7] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t d[8];
  int64_t br = 0;
  for (int i = 0; i < 8; ++i) {
    br += (int64_t)t[i] - FR_LIMBS[i];
    d[i] = (uint32_t)br;
    br >>= 32;
  }
  const bool keep_t = br < 0;
  for (int i = 0; i < 8; ++i) r.v[i] = keep_t ? t[i] : d[i];
}

BLS_HD BLS_INLINE bool fr_is_zero(const fr& a) {
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc |= a.v[i];
  return acc == 0;
}

BLS_HD BLS_INLINE void fr_from_u32(fr& r, uint32_t x) {
  fr t, r2;
  for (int i = 0; i < 8; ++i) {
    t.v[i] = i == 0 ? x : 0u;
    r2.v[i] = FR_R2[i];
  }
  fr_mul(r, t, r2);  // x < r so the product reduces
}

// A share index as herumi sets it: id.SetDecString(strconv.Itoa(idx)) (/root/reference/tbls/herumi.go:264-271)
// parses the decimal of a Go int, sign included, as an Fr element: idx mod r, so -k becomes r - k.
// |idx| < 2^63 < r, so the reduction is one conditional negation.  Result in Montgomery form.
BLS_HD BLS_INLINE void fr_from_i64(fr& r, int64_t x) {
  const uint64_t m = x < 0 ? (uint64_t)0 - (uint64_t)x : (uint64_t)x;
  fr t, r2;
  for (int i = 0; i < 8; ++i) {
    t.v[i] = i == 0 ? (uint32_t)m : (i == 1 ? (uint32_t)(m >> 32) : 0u);
    r2.v[i] = FR_R2[i];
  }
  fr_mul(r, t, r2);
  if (x < 0) {
    fr z;
    for (int i = 0; i < 8; ++i) z.v[i] = 0;
    fr_sub(r, z, r);
  }
}

BLS_HD BLS_INLINE void fr_to_plain(fr& r, const fr& a) {
  fr one;
  for (int i = 0; i < 8; ++i) one.v[i] = i == 0 ? 1u : 0u;
  fr_mul(r, a, one);
}


// Plain 32-byte big-endian scalar -> limbs; returns false when >= r
BLS_HD BLS_INLINE bool fr_plain_from_be32(fr& r, const uint8_t* b) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  int64_t br = 0;
  for (int i = 0; i < 8; ++i) {
    br += (int64_t)r.v[i] - FR_LIMBS[i];
    br >>= 32;
  }
  return br < 0;
}

BLS_HD BLS_CALL void fr_inv(fr& r, const fr& a) {
  fr acc = a;
  for (int i = 253; i >= 0; --i) {  // r - 2 has its top bit at 254
    fr_mul(acc, acc, acc);
    if ((FR_EXP_R_MINUS_2[i >> 5] >> (i & 31)) & 1u) fr_mul(acc, acc, a);
  }
  r = acc;
}

}  // namespace bls
