// Random-linear-combination BatchVerify (BASELINE configs[3]): the per-lane
// stages behind hipbls_batch_verify_rlc, written once for the HIP kernels and the host test build.
//
// Semantics: status[i] is exactly what tbls.Herumi.Verify (/root/reference/tbls/herumi.go:285-301)
// returns for item i.  Items are checked in windows of RLC_W consecutive items; a window passes
// when, with per-item 64-bit random scalars r_i,
//     prod_m e( sum_{i in window, msg i = m} r_i pk_i , H(m) ) * e( -g1 , sum_{i in window} r_i sig_i ) == 1
// (one multi-Miller loop, one final exponentiation per window).  Every sig and pk is decoded and
// subgroup-checked individually first, so a window that passes is valid item by item except with
// probability <= 2^-64 (standard small-exponent batch verification).  Items of a window that fails
// are re-verified individually (op_verify), so the bitmap never depends on the random scalars.
//
// Scalars: r_i = a_i + b_i * x  (x the BLS parameter, a_i, b_i uniform 32-bit) taken from
// SHA-256(seed || i).  The 2^64 values are distinct mod r, which is all the soundness argument
// needs, and both sides get the multiplication at half length through the endomorphisms:
//   G2: [r] sig = [a] sig + [b] psi(sig)       (psi = [x] on G2, curve.h g2_in_subgroup)
//   G1: [r] pk  = [a] pk  + [b] ([x] pk)       ([x] pk is the first half of the G1 subgroup test)
#pragma once
#include "ops.h"

namespace bls {

#ifndef RLC_W
#define RLC_W 8  // items per verdict window
#endif
constexpr int RLC_PENDING = -1;  // internal status: decoded fine, verdict not yet known

struct rlc_seed {
  uint32_t w[8];  // 32 seed bytes as big-endian words
};

// (a, b) = first 8 bytes of SHA-256(seed || be64(i))
BLS_HD BLS_INLINE void rlc_scalars(uint32_t& a, uint32_t& b, const rlc_seed& seed, uint64_t i) {
  uint32_t w[16];
  for (int k = 0; k < 8; ++k) w[k] = seed.w[k];
  w[8] = (uint32_t)(i >> 32);
  w[9] = (uint32_t)i;
  w[10] = 0x80000000u;
  for (int k = 11; k < 15; ++k) w[k] = 0;
  w[15] = 40 * 8;
  sha256_state s;
  sha256_init(s);
  sha256_compress(s, w);
  a = s.h[0];
  b = s.h[1];
}

// ---- SoA (limb-major) point storage: word k of element i at base[k * stride + i] -----------
template <int WORDS>
BLS_HD BLS_INLINE void soa_store(uint32_t* base, uint64_t stride, uint64_t i, const uint32_t* src) {
  for (int k = 0; k < WORDS; ++k) base[(uint64_t)k * stride + i] = src[k];
}
template <int WORDS>
BLS_HD BLS_INLINE void soa_load(uint32_t* dst, const uint32_t* base, uint64_t stride, uint64_t i) {
  for (int k = 0; k < WORDS; ++k) dst[k] = base[(uint64_t)k * stride + i];
}

// ---- AoS (point-major) storage: element i at base[WORDS * i ...], 16-byte aligned (WORDS % 4 == 0): for data a lane
// gathers by index, one element is WORDS / 4 contiguous 16-byte loads instead of WORDS scattered cache lines --------
template <int WORDS>
BLS_HD BLS_INLINE void aos_store(uint32_t* base, uint64_t i, const uint32_t* src) {
  static_assert(WORDS % 4 == 0, "16-byte groups");
#if defined(__HIP_DEVICE_COMPILE__)
  uint4* d = (uint4*)__builtin_assume_aligned(base + (uint64_t)WORDS * i, 16);
  for (int k = 0; k < WORDS / 4; ++k) d[k] = make_uint4(src[4 * k], src[4 * k + 1], src[4 * k + 2], src[4 * k + 3]);
#else
  for (int k = 0; k < WORDS; ++k) base[(uint64_t)WORDS * i + k] = src[k];
#endif
}
template <int WORDS>
BLS_HD BLS_INLINE void aos_load(uint32_t* dst, const uint32_t* base, uint64_t i) {
  static_assert(WORDS % 4 == 0, "16-byte groups");
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* s = (const uint4*)__builtin_assume_aligned(base + (uint64_t)WORDS * i, 16);
  for (int k = 0; k < WORDS / 4; ++k) {
    const uint4 v = s[k];
    dst[4 * k] = v.x;
    dst[4 * k + 1] = v.y;
    dst[4 * k + 2] = v.z;
    dst[4 * k + 3] = v.w;
  }
#else
  for (int k = 0; k < WORDS; ++k) dst[k] = base[(uint64_t)WORDS * i + k];
#endif
}

// [a] P + [b] Q with one shared doubling chain (Shamir's trick), 32-bit a, b
template <class F>
BLS_HD BLS_CALL void jac_mul2_u32(jac<F>& r, const jac<F>& P_in, const jac<F>& Q_in, uint32_t a, uint32_t b) {
  const jac<F> P = P_in;
  const jac<F> Q = Q_in;
  jac<F> PQ, acc, addend;
  jac_add(PQ, P, Q);
  jac_set_inf(acc);
  for (int bit = 31; bit >= 0; --bit) {
    jac<F> t;
    jac_dbl_body(t, acc);  // inlined doubling; acc's address is never taken, so it stays in registers
    acc = t;
    const uint32_t d = ((a >> bit) & 1u) | (((b >> bit) & 1u) << 1);
    addend = d == 1 ? P : (d == 2 ? Q : PQ);
    if (d) {
      jac<F> x = acc, y;
      jac_add_body(y, x, addend);  // inlined: no scratch round trip for the live accumulator per addition
      acc = y;
    }
  }
  r = acc;
}

// The same for affine P, Q with P + Q finite (sig and psi(sig) = [x] sig of a G2 point other than O): the three
// addends are made affine with one inversion, so every addition is mixed (7M + 4S instead of 11M + 5S in Fp2).
template <class F>
BLS_HD BLS_CALL void jac_mul2_u32_aff(jac<F>& r, const aff<F>& P, const aff<F>& Q, uint32_t a, uint32_t b) {
  aff<F> PQ;
  {
    jac<F> pj, pq;
    jac_from_aff(pj, P);
    jac_add_aff(pq, pj, Q);
    jac_to_aff(PQ, pq);
  }
  jac<F> acc;
  jac_set_inf(acc);
  for (int bit = 31; bit >= 0; --bit) {
    jac<F> t;
    jac_dbl_body(t, acc);
    acc = t;
    const uint32_t d = ((a >> bit) & 1u) | (((b >> bit) & 1u) << 1);
    const aff<F> addend = d == 1 ? P : (d == 2 ? Q : PQ);
    if (d) {
      jac<F> x = acc, y;
      jac_add_aff_body(y, x, addend);
      acc = y;
    }
  }
  r = acc;
}

// G1 decode with the subgroup test (phi(P) = [-x^2] P, as g1_in_subgroup) that also hands back
// [x] P, the half-way point of that test.
BLS_HD BLS_CALL int g1_decompress_keep_x(g1a& out, g1j& xP, const uint8_t* b) {
  const int st = g1_decompress(out, b, false);
  if (st != DEC_OK) return st;
  g1j p, q, q2, phi;
  jac_from_aff(p, out);
  jac_mul_u64(q, p, X_ABS);   // [|x|] P
  jac_mul_u64(q2, q, X_ABS);  // [x^2] P
  fp_mul(phi.x, p.x, FP_BETA);
  fp_neg(phi.y, p.y);
  phi.z = p.z;
  if (!jac_eq(q2, phi)) return DEC_BAD;
  jac_neg(xP, q);  // x < 0
  return DEC_OK;
}

// Stage 1 with the public key already decoded: dp = its DEC_* code, pk affine, xpk = [x] pk (from
// g1_decompress_keep_x, either just now or once at load time in the resident pubshare table).
// Decodes + subgroup-checks the signature in herumi's order, then stores [r_i] pk_i (G1 Jacobian,
// 36 words) and [r_i] sig_i (G2 Jacobian, 72 words).  Items that already have their final status
// (bad encoding, infinity) store the point at infinity.
BLS_HD BLS_CALL int rlc_item_decoded(int dp, const g1a& pk, const g1j& xpk, const uint8_t* sig96, const rlc_seed& seed,
                                     uint64_t i, uint32_t* rpk36, uint32_t* rsig72) {
  g1j rp;
  g2j rs;
  jac_set_inf(rp);
  jac_set_inf(rs);
  int st = RLC_PENDING;
  if (dp == DEC_BAD) st = HIPBLS_ERR_PUBKEY;
  g2a sig;
  if (st == RLC_PENDING) {
    const int ds = g2_decompress(sig, sig96, true);
    if (ds == DEC_BAD)
      st = HIPBLS_ERR_SIGNATURE;
    else if (dp == DEC_INF || ds == DEC_INF)
      st = HIPBLS_ERR_VERIFY;  // KeyValidate rejects the identity key; e(pk, H) != e(g1, O)
  }
  if (st == RLC_PENDING) {
    uint32_t a, b;
    rlc_scalars(a, b, seed, i);
    g1j pj;
    jac_from_aff(pj, pk);
    jac_mul2_u32(rp, pj, xpk, a, b);
    g2j sj, psj;
    jac_from_aff(sj, sig);
    g2_psi(psj, sj);  // = [x] sig for sig in G2 (checked above); Z stays 1
    g2a psa;
    psa.x = psj.x;
    psa.y = psj.y;
    jac_mul2_u32_aff(rs, sig, psa, a, b);
  }
  const uint32_t* p = &rp.x.v[0];
  for (int k = 0; k < 36; ++k) rpk36[k] = p[k];
  const uint32_t* s = &rs.x.c0.v[0];
  for (int k = 0; k < 72; ++k) rsig72[k] = s[k];
  return st;
}

// Stage 1, one lane per item, from the wire-format public key.
BLS_HD BLS_CALL int rlc_item(const uint8_t* pk48, const uint8_t* sig96, const rlc_seed& seed, uint64_t i,
                             uint32_t* rpk36, uint32_t* rsig72) {
  g1a pk;
  g1j xpk;
  const int dp = g1_decompress_keep_x(pk, xpk, pk48);
  return rlc_item_decoded(dp, pk, xpk, sig96, seed, i, rpk36, rsig72);
}

// ---- resident pubshare table: every pubshare decoded + subgroup-checked once ----
// SoA with stride T (table size): code[T] (DEC_*), then 24 words affine (x, y), then 36 words [x]pk.
constexpr int PUBTAB_WORDS = 24 + 36;

BLS_HD BLS_INLINE int pubtab_load_lane(uint64_t k, const uint8_t* pks, uint64_t T, int32_t* code, uint32_t* tab) {
  g1a pk;
  g1j xpk;
  const int dp = g1_decompress_keep_x(pk, xpk, pks + 48 * k);
  if (dp != DEC_OK) {
    fp_set_zero(pk.x);
    fp_set_zero(pk.y);
    jac_set_inf(xpk);
  }
  soa_store<24>(tab, T, k, &pk.x.v[0]);
  soa_store<36>(tab + 24 * T, T, k, &xpk.x.v[0]);
  code[k] = dp;
  return dp == DEC_BAD ? HIPBLS_ERR_PUBKEY : HIPBLS_OK;
}

BLS_HD BLS_INLINE int pubtab_get(g1a& pk, g1j& xpk, uint64_t k, uint64_t T, const int32_t* code, const uint32_t* tab) {
  soa_load<24>(&pk.x.v[0], tab, T, k);
  soa_load<36>(&xpk.x.v[0], tab + 24 * T, T, k);
  return code[k];
}

// tbls.Verify with the public key taken from the table (same statuses as op_verify); the Miller loop's f in LDS.
template <int S>
BLS_HD BLS_CALL int op_verify_decoded_pk(int dp, const g1a& pk, const uint8_t* msg, uint32_t msg_len,
                                         const uint8_t* sig96, const f12l<S> F) {
  if (dp == DEC_BAD) return HIPBLS_ERR_PUBKEY;
  g2a sig;
  const int ds = g2_decompress(sig, sig96, false);  // G2 membership from the Miller loop (ops.h)
  if (ds == DEC_BAD) return HIPBLS_ERR_SIGNATURE;
  if (dp == DEC_INF || ds == DEC_INF) return verify_inf_status(ds, sig);
  g2j hj;
  hash_to_g2(hj, msg, msg_len, DST_POP, 43);
  g2a hm;
  jac_to_aff(hm, hj);
  return pairing_check_verify_sig_l(pk, hm, sig, F);
}

// Multi-Miller loop over up to MAXN pairs with one shared Fp12 squaring chain (pairing.h steps).
template <int MAXN>
// T0_out (when given) receives the first pair's final T = [|x|] Q[0] (pairing.h g2_subgroup_from_miller).
BLS_HD BLS_CALL void miller_loop_multi(fp12& f, const g1a* P, const g2a* Q, int n, g2j* T0_out = nullptr) {
  g2j T[MAXN];
  for (int k = 0; k < n; ++k) {
    T[k].x = Q[k].x;
    T[k].y = Q[k].y;
    fp2_set_one(T[k].z);
  }
  fp12_set_one(f);
  fp2 g0, g1, h1;
  for (int bit = 62; bit >= 0; --bit) {
    if (bit != 62) fp12_sqr(f, f);
    // lines two at a time (fp12_mul_line2): one f update per pair of lines
    for (int k = 0; k < n; k += 2) {
      if (k + 1 < n) {
        fp2 a0, a1, ah;
        miller_dbl_step(T[k], a0, a1, ah, P[k].x, P[k].y);
        miller_dbl_step(T[k + 1], g0, g1, h1, P[k + 1].x, P[k + 1].y);
        fp12_mul_line2(f, a0, a1, ah, g0, g1, h1);
      } else {
        miller_dbl_step(T[k], g0, g1, h1, P[k].x, P[k].y);
        fp12_mul_line(f, g0, g1, h1);
      }
    }
    if ((X_ABS >> bit) & 1ull) {
      for (int k = 0; k < n; k += 2) {
        if (k + 1 < n) {
          fp2 a0, a1, ah;
          miller_add_step(T[k], a0, a1, ah, Q[k], P[k].x, P[k].y);
          miller_add_step(T[k + 1], g0, g1, h1, Q[k + 1], P[k + 1].x, P[k + 1].y);
          fp12_mul_line2(f, a0, a1, ah, g0, g1, h1);
        } else {
          miller_add_step(T[k], g0, g1, h1, Q[k], P[k].x, P[k].y);
          fp12_mul_line(f, g0, g1, h1);
        }
      }
    }
  }
  fp12_conj(f, f);
  if (T0_out) *T0_out = T[0];
}

// miller_loop_multi with f in LDS (pairing_lds.h): the same steps and the same f; T[] stays in the lane's stack.
template <int MAXN, int S>
BLS_HD BLS_CALL void miller_loop_multi_l(fp12& f_out, const f12l<S> F, const g1a* P, const g2a* Q, int n) {
  g2j T[MAXN];
  for (int k = 0; k < n; ++k) {
    T[k].x = Q[k].x;
    T[k].y = Q[k].y;
    fp2_set_one(T[k].z);
  }
  {
    fp12 one;
    fp12_set_one(one);
    F.st12(one);
  }
  fp2 g0, g1, h1;
  for (int bit = 62; bit >= 0; --bit) {
    if (bit != 62) fp12_sqr_l(F);
    for (int k = 0; k < n; k += 2) {
      if (k + 1 < n) {
        fp2 a0, a1, ah;
        miller_dbl_step(T[k], a0, a1, ah, P[k].x, P[k].y);
        miller_dbl_step(T[k + 1], g0, g1, h1, P[k + 1].x, P[k + 1].y);
        fp12_mul_line2_l(F, a0, a1, ah, g0, g1, h1);
      } else {
        miller_dbl_step(T[k], g0, g1, h1, P[k].x, P[k].y);
        fp12_mul_line_l(F, g0, g1, h1);
      }
    }
    if ((X_ABS >> bit) & 1ull) {
      for (int k = 0; k < n; k += 2) {
        if (k + 1 < n) {
          fp2 a0, a1, ah;
          miller_add_step(T[k], a0, a1, ah, Q[k], P[k].x, P[k].y);
          miller_add_step(T[k + 1], g0, g1, h1, Q[k + 1], P[k + 1].x, P[k + 1].y);
          fp12_mul_line2_l(F, a0, a1, ah, g0, g1, h1);
        } else {
          miller_add_step(T[k], g0, g1, h1, Q[k], P[k].x, P[k].y);
          fp12_mul_line_l(F, g0, g1, h1);
        }
      }
    }
  }
  fp12 f;
  F.ld12(f);
  fp12_conj(f_out, f);
}

// Stage 3, one lane per window [i0, i1): sum the scaled keys per run of equal message index and
// the scaled signatures over the whole window, run one multi-Miller loop + final exponentiation,
// and return true when the window verifies (or holds no pending item).
// Accessors are callables so the same body serves the SoA device buffers and the host test.
template <int LS, class LoadPk, class LoadSig, class LoadH>
BLS_HD BLS_INLINE bool rlc_window(const f12l<LS>& F, uint64_t i0, uint64_t i1, const int32_t* status, const uint32_t* msg_idx,
                                  LoadPk load_pk, LoadSig load_sig, LoadH load_h) {
  g1a P[RLC_W + 1];
  g2a Q[RLC_W + 1];
  int np = 0;
  g2j S;
  jac_set_inf(S);
  g1j run;
  uint32_t run_msg = 0xffffffffu;
  bool any = false;
  for (uint64_t i = i0; i < i1; ++i) {
    if (status[i] != RLC_PENDING) continue;
    any = true;
    g1j qp;
    g2j qs;
    load_pk(qp, i);
    load_sig(qs, i);
    jac_add(S, S, qs);
    const uint32_t m = msg_idx[i];
    if (m != run_msg) {
      if (run_msg != 0xffffffffu && !jac_is_inf(run)) {
        jac_to_aff(P[np], run);
        load_h(Q[np], run_msg);
        ++np;
      }
      run = qp;
      run_msg = m;
    } else {
      jac_add(run, run, qp);
    }
  }
  if (!any) return true;
  if (!jac_is_inf(run)) {
    jac_to_aff(P[np], run);
    load_h(Q[np], run_msg);
    ++np;
  }
  if (!jac_is_inf(S)) {
    P[np].x = G1_GEN_X;
    P[np].y = G1_NEG_GEN_Y;
    jac_to_aff(Q[np], S);
    ++np;
  }
  if (np == 0) return true;
  fp12 f;
  miller_loop_multi_l<RLC_W + 1>(f, F, P, Q, np);
  final_exp_l(f, f, F);  // in place (final_exponentiation_l allows r == f_in)
  return fp12_is_one(f);
}

// ---- lane bodies of the four stages (kernels in hipbls.hip; host loop in tests/native) --------

// Stage 1, item i: status (final, or RLC_PENDING) and the scaled pk / sig in SoA.
// pks == nullptr: the keys come from the resident table (key_idx[i] < T).
BLS_HD BLS_INLINE void rlc_items_lane(uint64_t i, const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx,
                                      uint64_t n, uint64_t n_msgs, const rlc_seed& seed, uint32_t* rpk,
                                      uint32_t* rsig, int32_t* status, const uint32_t* key_idx = nullptr,
                                      uint64_t T = 0, const int32_t* tcode = nullptr, const uint32_t* tab = nullptr) {
  uint32_t p[36], s[72];
  int st;
  if (msg_idx[i] >= n_msgs || (!pks && key_idx[i] >= T)) {  // device entry point: out-of-range index
    st = HIPBLS_ERR_ARG;
    g1j ip;
    g2j is;
    jac_set_inf(ip);
    jac_set_inf(is);
    for (int k = 0; k < 36; ++k) p[k] = (&ip.x.v[0])[k];
    for (int k = 0; k < 72; ++k) s[k] = (&is.x.c0.v[0])[k];
  } else if (pks) {
    st = rlc_item(pks + 48 * i, sigs + 96 * i, seed, i, p, s);
  } else {
    g1a pk;
    g1j xpk;
    const int dp = pubtab_get(pk, xpk, key_idx[i], T, tcode, tab);
    st = rlc_item_decoded(dp, pk, xpk, sigs + 96 * i, seed, i, p, s);
  }
  soa_store<36>(rpk, n, i, p);
  soa_store<72>(rsig, n, i, s);
  status[i] = st;
}

// H(m) table addressing: message m lives in column hslot[m] (the resident H(m) cache) or, with hslot == nullptr,
// in column m of a per-call table; the table has hstride columns of 48 words (affine, SoA).
BLS_HD BLS_INLINE uint64_t h_col(const uint32_t* hslot, uint64_t m) { return hslot ? (uint64_t)hslot[m] : m; }

// Stage 2, message m: H(m) in affine SoA (48 words) at its column.
BLS_HD BLS_INLINE void rlc_hash_lane(uint64_t m, const uint8_t* msgs, const uint64_t* offs, uint32_t* H,
                                     uint64_t hstride, const uint32_t* hslot) {
  const uint64_t o0 = offs[m], o1 = offs[m + 1];
  g2j hj;
  hash_to_g2(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43);
  g2a ha;
  jac_to_aff(ha, hj);
  soa_store<48>(H, hstride, h_col(hslot, m), &ha.x.c0.v[0]);
}

// Stage 3, window w = items [w*RLC_W, ...): on success every pending item becomes HIPBLS_OK,
// otherwise they stay pending for stage 4.  Returns (and stores in win_fail[w]) the number of items
// left pending: 0 when the window passed.
template <int S>
BLS_HD BLS_INLINE int rlc_window_lane(const f12l<S>& F, uint64_t w, uint64_t n, const uint32_t* msg_idx, const uint32_t* rpk,
                                      const uint32_t* rsig, const uint32_t* H, uint64_t hstride, const uint32_t* hslot,
                                      int32_t* status, int32_t* win_fail) {
  const uint64_t i0 = w * RLC_W;
  const uint64_t i1 = i0 + RLC_W < n ? i0 + RLC_W : n;
  auto load_pk = [&](g1j& q, uint64_t i) { soa_load<36>(&q.x.v[0], rpk, n, i); };
  auto load_sig = [&](g2j& q, uint64_t i) { soa_load<72>(&q.x.c0.v[0], rsig, n, i); };
  auto load_h = [&](g2a& q, uint32_t m) { soa_load<48>(&q.x.c0.v[0], H, hstride, h_col(hslot, m)); };
  const bool ok = rlc_window(F, i0, i1, status, msg_idx, load_pk, load_sig, load_h);
  int left = 0;
  for (uint64_t i = i0; i < i1; ++i)
    if (status[i] == RLC_PENDING) {
      if (ok)
        status[i] = HIPBLS_OK;
      else
        ++left;
    }
  win_fail[w] = left;
  return left;
}

// Stage 4, item i: still pending after its window failed -> tbls.Verify of the item alone.  Both
// points already passed decoding and the subgroup tests in stage 1 and H(m) is in the table, so this
// is the bare pairing check: e(pk, H(m)) * e(-g1, sig) == 1 (about half of a full op_verify).
// The fallback's points from stage 1 instead of the wire bytes: an item pending in a failed window has [r] pk and
// [r] sig stored (rlc_item_decoded; the batch-wide path's k_rlcb_mark stores the same), and for r != 0 mod the group
// order e([r] pk, H) == e(g1, [r] sig) exactly when e(pk, H) == e(g1, sig), so the re-check needs two inversions
// (to affine) instead of three square-root powers of decompression.  r = a + b x with a, b < 2^32 is 0 only for
// a = b = 0, which leaves both points at infinity: then (and without stored points) the caller decodes as before.
BLS_HD BLS_INLINE bool rlc_scaled_pair(g1a& pk, g2a& sig, const uint32_t* rpk, const uint32_t* rsig, uint64_t n,
                                       uint64_t i) {
  if (!rpk || !rsig) return false;
  g1j rp;
  g2j rs;
  soa_load<36>(&rp.x.v[0], rpk, n, i);
  soa_load<72>(&rs.x.c0.v[0], rsig, n, i);
  if (jac_is_inf(rp) || jac_is_inf(rs)) return false;
  jac_to_aff(pk, rp);
  jac_to_aff(sig, rs);
  return true;
}

template <int S>
BLS_HD BLS_INLINE void rlc_fallback_lane(const f12l<S>& F, uint64_t i, const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx,
                                         const uint32_t* H, uint64_t hstride, const uint32_t* hslot, int32_t* status,
                                         const uint32_t* key_idx = nullptr, uint64_t T = 0,
                                         const uint32_t* tab = nullptr, const uint32_t* rpk = nullptr,
                                         const uint32_t* rsig = nullptr, uint64_t n = 0) {
  if (status[i] != RLC_PENDING) return;
  g1a pk;
  g2a sig, hm;
  if (!rlc_scaled_pair(pk, sig, rpk, rsig, n, i)) {
    if (pks)
      g1_decompress(pk, pks + 48 * i, false);
    else
      soa_load<24>(&pk.x.v[0], tab, T, key_idx[i]);
    g2_decompress(sig, sigs + 96 * i, false);
  }
  soa_load<48>(&hm.x.c0.v[0], H, hstride, h_col(hslot, msg_idx[i]));
  status[i] = pairing_check_verify_l(pk, hm, sig, F) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
}

}  // namespace bls
