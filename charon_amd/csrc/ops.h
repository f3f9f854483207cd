// Per-item operations of the tbls.Implementation hot path, written once and called by the HIP
// kernels (one lane per item).  Status codes mirror the three error strings of
// tbls.Herumi.Verify (/root/reference/tbls/herumi.go:285-301):
//   HIPBLS_OK = 0, HIPBLS_ERR_PUBKEY = 1 ("cannot set compressed public key in Herumi format"),
//   HIPBLS_ERR_SIGNATURE = 2 ("cannot unmarshal signature into Herumi signature"),
//   HIPBLS_ERR_VERIFY = 3 ("signature not verified").
#pragma once
#include "../../include/hipbls.h"
#include "fr.h"
#include "h2c.h"
#include "pairing.h"
#include "pairing_lds.h"

namespace bls {

// Verify with pk and sig already decoded (affine, subgroup-checked) and H(m) already hashed.
BLS_HD BLS_CALL bool pairing_check_verify(const g1a& pk, const g2a& hm, const g2a& sig) {
  // e(pk, H(m)) * e(-g1, sig) == 1
  g1a P[2];
  g2a Q[2];
  bool skip[2] = {false, false};
  P[0] = pk;
  Q[0] = hm;
  P[1].x = G1_GEN_X;
  P[1].y = G1_NEG_GEN_Y;
  Q[1] = sig;
  fp12 f, e;
  miller_loop_n(f, P, Q, skip, 2);
  final_exponentiation(e, f);
  return fp12_is_one(e);
}

// The same check with the signature's G2 membership taken from the Miller loop's [|x|] sig (pairing.h
// g2_subgroup_from_miller) instead of a separate 63-doubling scalar multiplication.  sig is on the curve and not
// infinity.  Returns HIPBLS_OK, HIPBLS_ERR_SIGNATURE (sig not in G2: herumi's deserialization error, which wins over
// the pairing's verdict) or HIPBLS_ERR_VERIFY.
BLS_HD BLS_CALL int pairing_check_verify_sig(const g1a& pk, const g2a& hm, const g2a& sig) {
  g1a P1;
  P1.x = G1_GEN_X;
  P1.y = G1_NEG_GEN_Y;
  fp12 f, e;
  g2j T1;
  miller_loop_2(f, pk, hm, P1, sig, &T1);
  const bool in_g2 = g2_subgroup_from_miller(T1, sig);
  final_exponentiation(e, f);
  if (!in_g2) return HIPBLS_ERR_SIGNATURE;
  return fp12_is_one(e) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
}

// pairing_check_verify_sig with the Miller loop's f in LDS (pairing_lds.h): the C2 kernel k_verify_fused.
#ifndef BLS_VERIFY_L_CALL
#define BLS_VERIFY_L_CALL BLS_CALL
#endif
// INL: the Miller loop inlined here (k_verify_fused's kernel-inlined chain, op_verify_l_kernel) or called.
template <int S, bool INL>
BLS_HD BLS_INLINE int pairing_check_verify_sig_l_body(const g1a& pk, const g2a& hm, const g2a& sig, const f12l<S> F) {
  g1a P1;
  P1.x = G1_GEN_X;
  P1.y = G1_NEG_GEN_Y;
  fp12 f;
  bool in_g2;
  {
    g2j T1;
    if (INL)
      miller_loop_2_l_body<S, true>(f, F, pk, hm, P1, sig, &T1);
    else
      miller_loop_2_l<S, true>(f, F, pk, hm, P1, sig, &T1);
    in_g2 = g2_subgroup_from_miller(T1, sig);
  }
  final_exp_l(f, f, F);  // in place: one Fp12 less in this frame (final_exponentiation_l allows r == f_in)
  if (!in_g2) return HIPBLS_ERR_SIGNATURE;
  return fp12_is_one(f) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
}
template <int S>
BLS_HD BLS_VERIFY_L_CALL int pairing_check_verify_sig_l(const g1a& pk, const g2a& hm, const g2a& sig, const f12l<S> F) {
  return pairing_check_verify_sig_l_body<S, false>(pk, hm, sig, F);
}

// Statuses for the infinity cases (herumi: a valid infinity key or signature fails KeyValidate / the check), once the
// signature decoded with its membership still pending: a non-G2 signature is still a deserialization error.
BLS_HD BLS_INLINE int verify_inf_status(int ds, const g2a& sig) {
  if (ds == DEC_OK) {
    g2j sj;
    jac_from_aff(sj, sig);
    if (!g2_in_subgroup(sj)) return HIPBLS_ERR_SIGNATURE;
  }
  return HIPBLS_ERR_VERIFY;
}

// Full tbls.Verify for one item (used by the fused kernel and host-side instrumentation).

// sigma = sk * H(msg); returns HIPBLS_OK or HIPBLS_ERR_SECRET

// pk = sk * g1; zero secret is an error (GetSafePublicKey, herumi.go:74)

// Lagrange coefficient at 0 for the i-th id of a set: lambda_i = prod_{j != i} x_j / (x_j - x_i) over Fr, with
// x_k = ids[k] mod r (fr_from_i64: herumi's SetDecString(strconv.Itoa(idx)), tbls/herumi.go:264-271).  The ids
// must be non-zero and pairwise distinct (callers check; herumi's Recover fails otherwise).
BLS_HD BLS_CALL void lagrange_at_zero(fr& out_plain, const int64_t* ids, int n, int i) {
  fr num, den, t, xi, xj;
  fr_from_u32(num, 1);
  fr_from_u32(den, 1);
  fr_from_i64(xi, ids[i]);
  for (int j = 0; j < n; ++j) {
    if (j == i) continue;
    fr_from_i64(xj, ids[j]);
    fr_mul(num, num, xj);
    fr_sub(t, xj, xi);
    fr_mul(den, den, t);
  }
  fr_inv(den, den);
  fr_mul(t, num, den);
  fr_to_plain(out_plain, t);
}

// ThresholdAggregate with small share indices (charon's are 1..n, n the cluster size; app/app.go:344-381).
// lambda_k = N_k / D_k with the integers N_k = prod_{j != k} x_j and D_k = prod_{j != k} (x_j - x_k).  With
// L = lcm_k |D_k|, every c_k = N_k (L / D_k) is an integer and
//     sum_k lambda_k sig_k = [L^-1 mod r] sum_k c_k sig_k,
// so each partial needs a multiplication by a short integer (36 bits for 7-of-10 over ids 1..10) instead of a 255-bit
// lambda_k, and the group one 255-bit multiplication of the sum.  Returns false -- the caller takes the field path,
// lagrange_at_zero -- unless the whole group fits: t <= 16, |x_j| <= 2^20 and L and every c_k below 2^63.  The
// decision is the group's (every c_k is checked), so all lanes of a group and the group's sum agree on the path.
BLS_HD BLS_INLINE uint64_t gcd_u64(uint64_t a, uint64_t b) {
  while (b) {
    const uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}
BLS_HD BLS_CALL bool lagrange_small(const int64_t* ids, int t, int me, int64_t& c_me, uint64_t& L) {
  if (t < 1 || t > 16) return false;
  for (int a = 0; a < t; ++a)
    if (ids[a] > (1 << 20) || ids[a] < -(1 << 20) || ids[a] == 0) return false;
  int64_t D[16];
  uint64_t l = 1;
  for (int k = 0; k < t; ++k) {
    int64_t d = 1;
    for (int j = 0; j < t; ++j) {
      if (j == k) continue;
      if (__builtin_mul_overflow(d, ids[j] - ids[k], &d)) return false;
    }
    if (d == 0 || d == INT64_MIN) return false;  // duplicate ids (the status already says "cannot combine")
    D[k] = d;
    const uint64_t ad = d < 0 ? (uint64_t)(-d) : (uint64_t)d;
    if (__builtin_mul_overflow(l, ad / gcd_u64(l, ad), &l) || l > (uint64_t)INT64_MAX) return false;
  }
  for (int k = 0; k < t; ++k) {
    int64_t n = 1;
    for (int j = 0; j < t; ++j)
      if (j != k && __builtin_mul_overflow(n, ids[j], &n)) return false;
    const uint64_t ad = D[k] < 0 ? (uint64_t)(-D[k]) : (uint64_t)D[k];
    const int64_t f = D[k] < 0 ? -(int64_t)(l / ad) : (int64_t)(l / ad);
    int64_t c;
    if (__builtin_mul_overflow(n, f, &c) || c == INT64_MIN) return false;
    if (k == me) c_me = c;
  }
  L = l;
  return true;
}

// [c] P for a signed 64-bit c (jac_mul_u64 of |c|, negated for c < 0)
BLS_HD BLS_INLINE void g2_mul_i64(g2j& r, const g2j& p, int64_t c) {
  jac_mul_u64(r, p, c < 0 ? (uint64_t)0 - (uint64_t)c : (uint64_t)c);
  if (c < 0) {
    g2j t = r;
    jac_neg(r, t);
  }
}

// Partial k of a group (ids[0..t), this partial's index me): lambda_k * sig (small-integer path: c_k * sig, the
// group's sum is multiplied by L^-1 in tagg_unscale).
BLS_HD BLS_CALL void tagg_scale_point(g2j& out, const g2j& sj, const int64_t* ids, int t, int me) {
  int64_t c;
  uint64_t L;
  if (lagrange_small(ids, t, me, c, L)) {
    g2_mul_i64(out, sj, c);
  } else {
    fr lam;
    lagrange_at_zero(lam, ids, t, me);
    g2_mul_glv4(out, sj, lam.v);
  }
}

// A partial's G2 membership test and its small-integer multiple from ONE chain of doublings.  herumi deserializes
// every partial with a subgroup check (tbls/herumi.go:250-262), here psi(sig) == [x] sig (Scott 2021, as
// g2_in_subgroup), and the small-integer path then needs [c] sig.  Right to left, the points 2^i sig (i < 64) serve
// both: [|x|] sig = sum over |x|'s six set bits, [|c|] sig = sum over c's bits -- 63 doublings and ~23 additions
// instead of 63 + 35 doublings and the same additions.  The sums are the same group elements as the left-to-right
// chains compute (the additions handle the exceptional cases), so the aggregate's bytes do not change.  Returns
// whether sig is in G2 (sig affine, not infinity).
BLS_HD BLS_CALL bool g2_subgroup_and_mul_i64(g2j& out, const g2j& sj, int64_t c) {
  const uint64_t k = c < 0 ? (uint64_t)0 - (uint64_t)c : (uint64_t)c;
  g2j pw = sj, ax, ac;
  jac_set_inf(ax);
  jac_set_inf(ac);
  for (int i = 0; i < 64; ++i) {
    if ((X_ABS >> i) & 1ull) {  // wave-uniform, six times: the called addition
      g2j t = ax;
      jac_add(ax, t, pw);
    }
    if ((k >> i) & 1ull) {  // per lane, up to 64 times: inlined
      g2j t = ac;
      jac_add_body(ac, t, pw);
    }
    if (i < 63 && ((X_ABS | k) >> (i + 1)) != 0) {
      g2j t;
      jac_dbl_body(t, pw);
      pw = t;
    }
  }
  if (c < 0) {
    g2j t = ac;
    jac_neg(ac, t);
  }
  out = ac;
  g2j q, ps;
  jac_neg(q, ax);  // [x] sig, x < 0
  g2_psi(ps, sj);
  return jac_eq(q, ps);
}

// The group's sum of scaled partials -> the aggregate: [L^-1 mod r] sum on the small-integer path, as is otherwise.
BLS_HD BLS_CALL void tagg_unscale(g2j& acc, const int64_t* ids, int t) {
  int64_t c;
  uint64_t L;
  if (!lagrange_small(ids, t, 0, c, L) || jac_is_inf(acc)) return;
  fr lf, li, plain;
  fr_from_i64(lf, (int64_t)L);
  fr_inv(li, lf);
  fr_to_plain(plain, li);
  g2j x = acc;
  g2_mul_glv4(acc, x, plain.v);
}

// Aggregate-and-verify without waiting for [L^-1]: on the small-integer path the aggregate is sigma = [L^-1] S with
// S = sum_k c_k sig_k, and since L is invertible mod r,
//     e(pk, H(m)) == e(g1, [L^-1] S)   <=>   e([L] pk, H(m)) == e(g1, S)
// (raise both sides to L; G_T has order r).  So the pairing check runs on S and on [L] pk -- a G1 multiplication by
// an integer below 2^63 -- while [L^-1] S, which only the 96-byte output needs, runs beside it.  Returns 1 off the
// small-integer path (S is then sigma itself).
BLS_HD BLS_INLINE uint64_t tagg_group_L(const int64_t* ids, int t) {
  int64_t c;
  uint64_t L;
  return lagrange_small(ids, t, 0, c, L) ? L : 1;
}
// pk <- [L] pk for pk in G1, not infinity: [L] pk is not infinity either (0 < L < 2^63 < r).
BLS_HD BLS_CALL void g1_scale_affine(g1a& pk, uint64_t L) {
  if (L <= 1) return;
  g1j pj, q;
  jac_from_aff(pj, pk);
  jac_mul_u64(q, pj, L);
  jac_to_aff(pk, q);
}

// One ThresholdAggregate group on one lane (host builds: tests/native): status as the kernels'.
BLS_HD BLS_CALL int op_threshold_aggregate(uint8_t* out96, const uint8_t* sigs, const int64_t* ids, int t) {
  int st = t > 0 ? HIPBLS_OK : HIPBLS_ERR_COMBINE;
  for (int a = 0; a < t; ++a) {
    if (ids[a] == 0) st = HIPBLS_ERR_COMBINE;
    for (int b = a + 1; b < t; ++b)
      if (ids[a] == ids[b]) st = HIPBLS_ERR_COMBINE;
  }
  g2j acc;
  jac_set_inf(acc);
  for (int k = 0; k < t; ++k) {  // every partial is deserialized first (herumi.go:250-262)
    g2a s;
    const int ds = g2_decompress(s, sigs + 96 * k, true);
    if (ds == DEC_BAD) return HIPBLS_ERR_SIGNATURE;
    if (st != HIPBLS_OK || ds == DEC_INF) continue;
    g2j sj, p;
    jac_from_aff(sj, s);
    tagg_scale_point(p, sj, ids, t, k);
    g2j x = acc;
    jac_add(acc, x, p);
  }
  if (st != HIPBLS_OK) return st;
  tagg_unscale(acc, ids, t);
  g2_compress(out96, acc);
  return HIPBLS_OK;
}

BLS_HD BLS_CALL int op_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t msg_len, const uint8_t* sig96) {
  g1a pk;
  const int dp = g1_decompress(pk, pk48, true);
  if (dp == DEC_BAD) return HIPBLS_ERR_PUBKEY;
  g2a sig;
  const int ds = g2_decompress(sig, sig96, false);  // G2 membership: from the Miller loop below
  if (ds == DEC_BAD) return HIPBLS_ERR_SIGNATURE;
  if (dp == DEC_INF || ds == DEC_INF) return verify_inf_status(ds, sig);  // KeyValidate / e(pk,H) != 1
  g2j hj;
  hash_to_g2(hj, msg, msg_len, DST_POP, 43);
  g2a hm;
  jac_to_aff(hm, hj);
  return pairing_check_verify_sig(pk, hm, sig);
}

// op_verify with the Miller loop's f in LDS (F: this lane's slot; pairing_lds.h).
template <int S, bool INL>
BLS_HD BLS_INLINE int op_verify_l_body(const uint8_t* pk48, const uint8_t* msg, uint32_t msg_len, const uint8_t* sig96,
                                     const f12l<S> F) {
  g1a pk;
  const int dp = g1_decompress(pk, pk48, true);
  if (dp == DEC_BAD) return HIPBLS_ERR_PUBKEY;
  g2a sig;
  const int ds = g2_decompress(sig, sig96, false);
  if (ds == DEC_BAD) return HIPBLS_ERR_SIGNATURE;
  if (dp == DEC_INF || ds == DEC_INF) return verify_inf_status(ds, sig);
  g2j hj;
  hash_to_g2(hj, msg, msg_len, DST_POP, 43);
  g2a hm;
  jac_to_aff(hm, hj);
  return pairing_check_verify_sig_l_body<S, INL>(pk, hm, sig, F);
}
template <int S>
BLS_HD BLS_VERIFY_L_CALL int op_verify_l(const uint8_t* pk48, const uint8_t* msg, uint32_t msg_len, const uint8_t* sig96,
                                const f12l<S> F) {
  return op_verify_l_body<S, false>(pk48, msg, msg_len, sig96, F);
}
// k_verify_fused's form: the whole chain down to the Miller loop inlined into the kernel (pairing_lds.h
// miller_loop_2_l_body); the final exponentiation and the other callees stay out of line.
template <int S>
BLS_HD BLS_INLINE int op_verify_l_kernel(const uint8_t* pk48, const uint8_t* msg, uint32_t msg_len, const uint8_t* sig96,
                                         const f12l<S> F) {
  return op_verify_l_body<S, true>(pk48, msg, msg_len, sig96, F);
}

BLS_HD BLS_CALL int op_sign(uint8_t* out96, const uint8_t* sk32, const uint8_t* msg, uint32_t msg_len) {
  fr sk;
  if (!fr_plain_from_be32(sk, sk32)) return HIPBLS_ERR_SECRET;
  g2j h, s;
  hash_to_g2(h, msg, msg_len, DST_POP, 43);
  g2_mul_glv4(s, h, sk.v);
  g2_compress(out96, s);
  return HIPBLS_OK;
}

BLS_HD BLS_CALL int op_sk_to_pk(uint8_t* out48, const uint8_t* sk32) {
  fr sk;
  if (!fr_plain_from_be32(sk, sk32)) return HIPBLS_ERR_SECRET;
  if (fr_is_zero(sk)) return HIPBLS_ERR_SECRET;
  g1j g, pk;
  g.x = G1_GEN_X;
  g.y = G1_GEN_Y;
  fp_set_one(g.z);
  jac_mul_limbs(pk, g, sk.v, 8);
  g1_compress(out48, pk);
  return HIPBLS_OK;
}

}  // namespace bls
