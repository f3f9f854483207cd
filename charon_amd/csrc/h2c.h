// hash_to_curve for G2, ciphersuite BLS12381G2_XMD:SHA-256_SSWU_RO_ (RFC 9380), the map herumi's
// EthModeLatest applies to every signing root before the pairing check
// (/root/reference/tbls/herumi.go:29-33, :298 VerifyByte).  One lane hashes one message:
//   expand_message_xmd (SHA-256, 256 bytes) -> 2 Fp2 field elements -> simplified SWU on the
//   3-isogenous curve E2' -> 3-isogeny to E2 -> add -> clear cofactor via psi (RFC 9380 G.3).
#pragma once
#include "curve.h"

namespace bls {

// The POP ciphersuite DST (43 bytes) used by Eth2 / herumi EthModeLatest.
static constexpr uint8_t DST_POP[43] = {'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8',
                                        '1', 'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6',
                                        '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

// ---------------------------------------------------------------------------------- SHA-256
struct sha256_state {
  uint32_t h[8];
};

BLS_HD BLS_INLINE uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }


BLS_HD BLS_INLINE void sha256_init(sha256_state& s) {
  s.h[0] = 0x6a09e667u;
  s.h[1] = 0xbb67ae85u;
  s.h[2] = 0x3c6ef372u;
  s.h[3] = 0xa54ff53au;
  s.h[4] = 0x510e527fu;
  s.h[5] = 0x9b05688cu;
  s.h[6] = 0x1f83d9abu;
  s.h[7] = 0x5be0cd19u;
}

// A message presented as up to four concatenated byte segments, hashed without materializing it.
struct byte_segs {
  const uint8_t* p[4];
  uint32_t n[4];
};

BLS_HD BLS_INLINE uint8_t segs_byte(const byte_segs& m, uint32_t pos) {
  for (int k = 0; k < 4; ++k) {
    if (pos < m.n[k]) return m.p[k] ? m.p[k][pos] : (uint8_t)0;
    pos -= m.n[k];
  }
  return 0;
}

// Full SHA-256 over the concatenation; out = 32-byte digest as 8 big-endian words.

// expand_message_xmd(msg, DST, 256) -> 64 big-endian words

// 64 uniform bytes (16 big-endian words) -> Fp element (Montgomery form), value mod p

BLS_HD BLS_INLINE int fp2_sgn0(const fp2& a) {
  fp t0, t1;
  fp_from_mont(t0, a.c0);
  fp_from_mont(t1, a.c1);
  const int s0 = (int)(t0.v[0] & 1u);
  const int z0 = fp_is_zero(t0) ? 1 : 0;
  const int s1 = (int)(t1.v[0] & 1u);
  return s0 | (z0 & s1);
}

// simplified SWU onto E2': y^2 = x^3 + A'x + B' (RFC 9380 6.6.2, straight-line form)
// 3-isogeny E2' -> E2, returning Jacobian coordinates (no inversion)
// full hash_to_curve; result in Jacobian coordinates on E2 (in G2)

BLS_HD BLS_CALL void sha256_compress(sha256_state& s, const uint32_t w_in[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = w_in[i];
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K[i] + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
  s.h[5] += f;
  s.h[6] += g;
  s.h[7] += h;
}

BLS_HD BLS_CALL void sha256_segs(uint32_t out[8], const byte_segs& m) {
  const uint32_t len = m.n[0] + m.n[1] + m.n[2] + m.n[3];
  const uint32_t nblocks = (len + 9 + 63) / 64;
  sha256_state s;
  sha256_init(s);
  for (uint32_t blk = 0; blk < nblocks; ++blk) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) {
      uint32_t word = 0;
      for (int k = 0; k < 4; ++k) {
        const uint32_t pos = blk * 64 + 4 * i + k;
        uint8_t byte;
        if (pos < len)
          byte = segs_byte(m, pos);
        else if (pos == len)
          byte = 0x80;
        else if (pos >= nblocks * 64 - 8) {
          const uint64_t bits = (uint64_t)len * 8;
          const int sh = (int)(nblocks * 64 - 1 - pos) * 8;
          byte = (uint8_t)(bits >> sh);
        } else
          byte = 0;
        word = (word << 8) | byte;
      }
      w[i] = word;
    }
    sha256_compress(s, w);
  }
  for (int i = 0; i < 8; ++i) out[i] = s.h[i];
}

BLS_HD BLS_INLINE uint32_t be32(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return (a << 24) | (b << 16) | (c << 8) | d;
}

// expand_message_xmd_256 for a 32-byte message (a signing root) and a 43-byte DST (the POP suite's): every byte's
// block and position is a compile-time constant, so the blocks are assembled as words in registers.  msg_prime is
// 143 bytes (Z_pad, msg, 0x01 0x00 0x00, DST, 43): three blocks, the first all zero; each b_i message is 77 bytes
// ((b_0 ^ b_(i-1)), i, DST, 43): two blocks.  18 compressions from words, no byte arrays (the general form below
// assembles every block byte by byte from segment lists in scratch: 266 -> <60 us at the n = 1 placement,
// charon_amd/tools/lat_parts_probe.hip).  Same output as the general form (tests/test_host_arith.py).
BLS_HD BLS_CALL void expand_message_xmd_256_m32_d43(uint32_t out[64], const uint8_t* msg, const uint8_t* dst) {
  uint32_t D[44];
#pragma unroll
  for (int i = 0; i < 43; ++i) D[i] = dst[i];
  D[43] = 43;
  uint32_t mw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mw[i] = be32(msg[4 * i], msg[4 * i + 1], msg[4 * i + 2], msg[4 * i + 3]);
  uint32_t w[16];
  sha256_state s;
  sha256_init(s);
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = 0;
  sha256_compress(s, w);  // Z_pad
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = mw[i];
  w[8] = be32(0x01, 0x00, 0x00, D[0]);
#pragma unroll
  for (int i = 9; i < 16; ++i) w[i] = be32(D[4 * i - 35], D[4 * i - 34], D[4 * i - 33], D[4 * i - 32]);  // D[1..28]
  sha256_compress(s, w);
  w[0] = be32(D[29], D[30], D[31], D[32]);
  w[1] = be32(D[33], D[34], D[35], D[36]);
  w[2] = be32(D[37], D[38], D[39], D[40]);
  w[3] = be32(D[41], D[42], D[43], 0x80);
#pragma unroll
  for (int i = 4; i < 15; ++i) w[i] = 0;
  w[15] = 143 * 8;
  sha256_compress(s, w);
  uint32_t b0[8], prev[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    b0[i] = s.h[i];
    prev[i] = 0;
  }
  // the b_i messages' DST words: block 1 ends with D[0..30] after (x, i); block 2 holds D[31..43] and the padding
  uint32_t t1[7], t2[4];
#pragma unroll
  for (int i = 0; i < 7; ++i) t1[i] = be32(D[4 * i + 3], D[4 * i + 4], D[4 * i + 5], D[4 * i + 6]);  // D[3..30]
  t2[0] = be32(D[31], D[32], D[33], D[34]);
  t2[1] = be32(D[35], D[36], D[37], D[38]);
  t2[2] = be32(D[39], D[40], D[41], D[42]);
  t2[3] = be32(D[43], 0x80, 0, 0);
#pragma unroll 1
  for (int idx = 1; idx <= 8; ++idx) {
    sha256_init(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = b0[i] ^ prev[i];
    w[8] = be32((uint32_t)idx, D[0], D[1], D[2]);
#pragma unroll
    for (int i = 0; i < 7; ++i) w[9 + i] = t1[i];
    sha256_compress(s, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = t2[i];
#pragma unroll
    for (int i = 4; i < 15; ++i) w[i] = 0;
    w[15] = 77 * 8;
    sha256_compress(s, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      prev[i] = s.h[i];
      out[(idx - 1) * 8 + i] = s.h[i];
    }
  }
}

BLS_HD BLS_CALL void expand_message_xmd_256(uint32_t out[64], const uint8_t* msg, uint32_t msg_len,
                                                const uint8_t* dst, uint32_t dst_len) {
  if (msg_len == 32 && dst_len == 43) {
    expand_message_xmd_256_m32_d43(out, msg, dst);
    return;
  }
  // msg_prime = Z_pad(64) || msg || I2OSP(256, 2) || I2OSP(0, 1) || DST || I2OSP(len(DST), 1)
  uint8_t mid[3] = {0x01, 0x00, 0x00};  // l_i_b_str = 0x0100, then 0x00
  uint8_t dst_tail[1] = {(uint8_t)dst_len};
  byte_segs m0;
  m0.p[0] = nullptr;
  m0.n[0] = 64;
  m0.p[1] = msg;
  m0.n[1] = msg_len;
  m0.p[2] = mid;
  m0.n[2] = 3;
  m0.p[3] = dst;
  m0.n[3] = dst_len;
  // dst_prime's trailing length byte is appended by making the last segment one longer: handled by
  // hashing DST then tail -- byte_segs holds 4 segments, so fold the tail into a local copy.
  uint8_t dstp[256];
  for (uint32_t i = 0; i < dst_len; ++i) dstp[i] = dst[i];
  dstp[dst_len] = dst_tail[0];
  m0.p[3] = dstp;
  m0.n[3] = dst_len + 1;
  uint32_t b0[8];
  sha256_segs(b0, m0);
  uint8_t b0b[32], prev[32];
  for (int i = 0; i < 8; ++i) {
    b0b[4 * i] = (uint8_t)(b0[i] >> 24);
    b0b[4 * i + 1] = (uint8_t)(b0[i] >> 16);
    b0b[4 * i + 2] = (uint8_t)(b0[i] >> 8);
    b0b[4 * i + 3] = (uint8_t)b0[i];
  }
  for (int i = 0; i < 32; ++i) prev[i] = 0;  // b_0 xor b_0... b_1 uses b_0 directly (prev = 0)
  for (int idx = 1; idx <= 8; ++idx) {
    uint8_t x[32];
    for (int i = 0; i < 32; ++i) x[i] = b0b[i] ^ prev[i];
    uint8_t ib[1] = {(uint8_t)idx};
    byte_segs m;
    m.p[0] = x;
    m.n[0] = 32;
    m.p[1] = ib;
    m.n[1] = 1;
    m.p[2] = dstp;
    m.n[2] = dst_len + 1;
    m.p[3] = nullptr;
    m.n[3] = 0;
    uint32_t bi[8];
    sha256_segs(bi, m);
    for (int i = 0; i < 8; ++i) {
      out[(idx - 1) * 8 + i] = bi[i];
      prev[4 * i] = (uint8_t)(bi[i] >> 24);
      prev[4 * i + 1] = (uint8_t)(bi[i] >> 16);
      prev[4 * i + 2] = (uint8_t)(bi[i] >> 8);
      prev[4 * i + 3] = (uint8_t)bi[i];
    }
  }
}

BLS_HD BLS_CALL void fp_from_be64_words(fp& r, const uint32_t* w) {
  // X = X_hi * 2^256 + X_lo with X_hi, X_lo < 2^256 < p;  mont(X) = mont_mul(X_lo, R^2) + mont_mul(X_hi, 2^256 R^2)
  fp hi, lo, c;
  for (int i = 0; i < 12; ++i) {
    hi.v[i] = 0;
    lo.v[i] = 0;
  }
  for (int i = 0; i < 8; ++i) {
    hi.v[i] = w[7 - i];
    lo.v[i] = w[15 - i];
  }
  for (int i = 0; i < 12; ++i) c.v[i] = R2_LIMBS[i];
  fp_mul(lo, lo, c);
  for (int i = 0; i < 12; ++i) c.v[i] = R2_2_256_LIMBS[i];
  fp_mul(hi, hi, c);
  fp_add(r, lo, hi);
}

// SSWU denominator: zu2 = Z u^2, den = zu2^2 + zu2
BLS_HD BLS_INLINE void sswu_den(fp2& zu2, fp2& den, const fp2& u) {
  fp2 u2;
  fp2_sqr(u2, u);
  fp2_mul(zu2, SSWU_Z, u2);
  fp2_sqr(den, zu2);
  fp2_add(den, den, zu2);
}
// SSWU with tv1 = inv0(den) supplied by the caller (so hash_to_g2 can share one inversion)
BLS_HD BLS_CALL void map_to_curve_sswu_tv(g2a& out, const fp2& u_in, const fp2& zu2_in, const fp2& tv1_in) {
  const fp2 u = u_in;
  const fp2 zu2 = zu2_in;
  const fp2 tv1 = tv1_in;
  fp2 x1, gx1, t, y, x;
  if (fp2_is_zero(tv1)) {
    x1 = SSWU_B_OVER_ZA;
  } else {
    fp2 one;
    fp2_set_one(one);
    fp2_add(t, one, tv1);
    fp2_mul(x1, SSWU_NEG_B_OVER_A, t);
  }
  // gx1 = x1^3 + A x1 + B, and the second candidate x2 = Z u^2 x1, gx2 = x2^3 + A x2 + B
  fp2_sqr(gx1, x1);
  fp2_mul(gx1, gx1, x1);
  fp2_mul(t, SSWU_A, x1);
  fp2_add(gx1, gx1, t);
  fp2_add(gx1, gx1, SSWU_B);
  fp2 x2, gx2;
  fp2_mul(x2, zu2, x1);
  fp2_sqr(gx2, x2);
  fp2_mul(gx2, gx2, x2);
  fp2_mul(t, SSWU_A, x2);
  fp2_add(gx2, gx2, t);
  fp2_add(gx2, gx2, SSWU_B);
  // One exponentiation decides and roots both (RFC 9380 6.6.2 picks x1 iff gx1 is square; any root of the chosen
  // g(x) serves, the sign is fixed below).  a in Fp2 is a square iff N(a) is a square in Fp (p = 3 mod 4), and
  // s = N(gx1)^((p+1)/4) has s^2 = N(gx1) or -N(gx1).  When gx1 is not a square, tv1 != 0 (g(B/(ZA)) is square
  // by the choice of Z), so gx2 = (Z u^2)^3 gx1 and N(gx2) = N(u)^6 (-N(Z)^3) (-N(gx1)) has the root
  // N(u)^3 sqrt(-N(Z)^3) s.  The Fp2 root then costs one more exponentiation instead of two per candidate, and no
  // lane of a wave waits on a second candidate's branch.
  fp n1, s, s2, nu, q;
  fp_sqr(n1, gx1.c0);
  fp_sqr(q, gx1.c1);
  fp_add(n1, n1, q);
  fp_pow(s, n1, EXP_SQRT, 378);
  fp_sqr(s2, s);
  const bool gx1_square = fp_eq(s2, n1);
  fp_sqr(nu, u.c0);
  fp_sqr(q, u.c1);
  fp_add(nu, nu, q);
  fp_sqr(q, nu);
  fp_mul(q, q, nu);
  fp_mul(q, q, SSWU_SQRT_NEG_NZ3);
  fp_mul(q, q, s);
  fp2 w;
  fp sw;
  if (gx1_square) {
    x = x1;
    w = gx1;
    sw = s;
  } else {
    x = x2;
    w = gx2;
    sw = q;
  }
  fp2_sqrt_from_norm_root(y, w, sw);
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  out.x = x;
  out.y = y;
}
BLS_HD BLS_CALL void map_to_curve_sswu(g2a& out, const fp2& u) {
  fp2 zu2, den, tv1;
  sswu_den(zu2, den, u);
  fp2_inv(tv1, den);  // inv0: 0 -> 0
  map_to_curve_sswu_tv(out, u, zu2, tv1);
}

BLS_HD BLS_CALL void iso_map_g2(g2j& out, const g2a& p_in) {
  const g2a p = p_in;
  // x = xn/xd, y = y * yn/yd  ->  Jacobian (xn xd yd^2, y yn xd^3 yd^2, xd yd)
  const fp2& x = p.x;
  fp2 xn, xd, yn, yd, t;
  xn = ISO_XNUM[3];
  for (int i = 2; i >= 0; --i) {
    fp2_mul(xn, xn, x);
    fp2_add(xn, xn, ISO_XNUM[i]);
  }
  fp2_add(xd, x, ISO_XDEN[1]);  // monic: x^2 + k1 x + k0
  fp2_mul(xd, xd, x);
  fp2_add(xd, xd, ISO_XDEN[0]);
  yn = ISO_YNUM[3];
  for (int i = 2; i >= 0; --i) {
    fp2_mul(yn, yn, x);
    fp2_add(yn, yn, ISO_YNUM[i]);
  }
  fp2_add(yd, x, ISO_YDEN[2]);  // monic cubic
  fp2_mul(yd, yd, x);
  fp2_add(yd, yd, ISO_YDEN[1]);
  fp2_mul(yd, yd, x);
  fp2_add(yd, yd, ISO_YDEN[0]);
  fp2 z, z2, xd2;
  fp2_mul(z, xd, yd);      // Z
  fp2_mul(t, z, yd);       // xd yd^2
  fp2_mul(out.x, xn, t);   // X = xn xd yd^2
  fp2_sqr(xd2, xd);
  fp2_mul(z2, t, xd2);     // xd^3 yd^2
  fp2_mul(t, p.y, yn);
  fp2_mul(out.y, t, z2);   // Y = y yn xd^3 yd^2
  out.z = z;
}

BLS_HD BLS_CALL void hash_to_g2(g2j& out, const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                                    uint32_t dst_len) {
  uint32_t uni[64];
  expand_message_xmd_256(uni, msg, msg_len, dst, dst_len);
  fp2 u0, u1;
  fp_from_be64_words(u0.c0, uni + 0);
  fp_from_be64_words(u0.c1, uni + 16);
  fp_from_be64_words(u1.c0, uni + 32);
  fp_from_be64_words(u1.c1, uni + 48);
  // both SSWU inversions from one (Montgomery's trick); a zero denominator keeps inv0 semantics
  // through separate inversions (fp2_inv(0) = 0)
  fp2 zu0, zu1, d0, d1, t0, t1, inv;
  sswu_den(zu0, d0, u0);
  sswu_den(zu1, d1, u1);
  fp2_mul(inv, d0, d1);
  if (fp2_is_zero(inv)) {
    fp2_inv(t0, d0);
    fp2_inv(t1, d1);
  } else {
    fp2_inv(inv, inv);
    fp2_mul(t0, inv, d1);
    fp2_mul(t1, inv, d0);
  }
  g2a q0a, q1a;
  map_to_curve_sswu_tv(q0a, u0, zu0, t0);
  map_to_curve_sswu_tv(q1a, u1, zu1, t1);
  g2j q0, q1, s;
  iso_map_g2(q0, q0a);
  iso_map_g2(q1, q1a);
  jac_add(s, q0, q1);
  g2_clear_cofactor(out, s);
}

}  // namespace bls
