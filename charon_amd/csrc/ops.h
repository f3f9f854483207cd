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
