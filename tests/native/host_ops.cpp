// Host (x86) build of the HIP engine's per-lane arithmetic (charon_amd/csrc/*.h), exported for
// ctypes so tests/test_host_arith.py can diff every layer against oracle/bls12381.py without a GPU.
// TEST INFRASTRUCTURE ONLY: the product library (charon_amd/libhipbls.so) never calls this code;
// it is the same source compiled for the CPU so kernel bugs show up in the CPU test suite.
#define BLS_COUNT_OPS 1
#include "../../charon_amd/csrc/ops.h"

static uint64_t g_rlcb_slots = 0;   // device wave slots rlcb_chunk_count plans for (ht_rlcb_set_slots)
static uint64_t g_rlcb_chunks = 0;  // test override of the chunk count (0: rlcb_chunk_count)
static uint32_t g_g1m_min = 64;     // G1 MSM threshold (ht_rlcb_set_g1_min; the device's hipbls_rlc_set_g1_msm_min)
namespace bls {
thread_local uint64_t g_fp_mul_count = 0;
thread_local uint64_t g_fp_sqr_count = 0;
#if defined(BLS_CONTRACT_CHECK)
uint64_t g_contract_violations = 0;
const char* g_contract_first = nullptr;
uint64_t g_contract_lazy_operands = 0;
#endif
}  // namespace bls
#if defined(BLS_CONTRACT_CHECK)
// operand-contract violations counted by the BLS_CONTRACT_CHECK build (field.h), and the first one's description
extern "C" uint64_t ht_contract_violations(void) { return bls::g_contract_violations; }
extern "C" const char* ht_contract_first(void) { return bls::g_contract_first; }
extern "C" uint64_t ht_contract_lazy_operands(void) { return bls::g_contract_lazy_operands; }
#endif

using namespace bls;

static void fp_out(uint8_t* o, const fp& a) {
  fp t;
  fp_from_mont(t, a);
  fp_plain_to_be48(o, t);
}
static void fp_in(fp& a, const uint8_t* b) {
  fp_plain_from_be48(a, b);
  fp_to_mont(a, a);
}

// The host stand-in for a lane's LDS slot of the Miller-loop f (pairing_lds.h, S = 1)
static f12l<1> host_f12_slot() {
  static thread_local u32x4 slot[36];
  return f12l<1>{slot};
}

extern "C" {

int ht_sign(const uint8_t* sk, const uint8_t* msg, uint32_t len, uint8_t* out) { return op_sign(out, sk, msg, len); }
int ht_sk_to_pk(const uint8_t* sk, uint8_t* out) { return op_sk_to_pk(out, sk); }
int ht_verify(const uint8_t* pk, const uint8_t* msg, uint32_t len, const uint8_t* sig) {
  return op_verify(pk, msg, len, sig);
}
// op_verify_l (k_verify_fused's path: the Miller loop's f in LDS, pairing_lds.h) over a host array standing in for
// the lane's LDS slot (one lane: S = 1)
int ht_verify_l(const uint8_t* pk, const uint8_t* msg, uint32_t len, const uint8_t* sig) {
  u32x4 slot[36];
  const f12l<1> F{slot};
  return op_verify_l(pk, msg, len, sig, F);
}

void ht_hash_to_g2(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dst_len, uint8_t* out_aff192) {
  g2j h;
  hash_to_g2(h, msg, len, dst, dst_len);
  g2a a;
  jac_to_aff(a, h);
  fp_out(out_aff192, a.x.c0);
  fp_out(out_aff192 + 48, a.x.c1);
  fp_out(out_aff192 + 96, a.y.c0);
  fp_out(out_aff192 + 144, a.y.c1);
}

void ht_expand_message(const uint8_t* msg, uint32_t len, const uint8_t* dst, uint32_t dst_len, uint8_t* out256) {
  uint32_t w[64];
  expand_message_xmd_256(w, msg, len, dst, dst_len);
  for (int i = 0; i < 64; ++i) {
    out256[4 * i] = (uint8_t)(w[i] >> 24);
    out256[4 * i + 1] = (uint8_t)(w[i] >> 16);
    out256[4 * i + 2] = (uint8_t)(w[i] >> 8);
    out256[4 * i + 3] = (uint8_t)w[i];
  }
}

// u (plain c0||c1) -> SSWU point on E2' (plain x0,x1,y0,y1)
void ht_map_to_curve(const uint8_t* u96, uint8_t* out192) {
  fp2 u;
  fp_in(u.c0, u96);
  fp_in(u.c1, u96 + 48);
  g2a p;
  map_to_curve_sswu(p, u);
  fp_out(out192, p.x.c0);
  fp_out(out192 + 48, p.x.c1);
  fp_out(out192 + 96, p.y.c0);
  fp_out(out192 + 144, p.y.c1);
}

int ht_g1_decompress(const uint8_t* in, int check, uint8_t* out96) {
  g1a a;
  int st = g1_decompress(a, in, check != 0);
  if (st == DEC_OK) {
    fp_out(out96, a.x);
    fp_out(out96 + 48, a.y);
  }
  return st;
}
int ht_g2_decompress(const uint8_t* in, int check, uint8_t* out192) {
  g2a a;
  int st = g2_decompress(a, in, check != 0);
  if (st == DEC_OK) {
    fp_out(out192, a.x.c0);
    fp_out(out192 + 48, a.x.c1);
    fp_out(out192 + 96, a.y.c0);
    fp_out(out192 + 144, a.y.c1);
  }
  return st;
}
int ht_g1_in_subgroup(const uint8_t* xy96) {
  g1j p;
  fp_in(p.x, xy96);
  fp_in(p.y, xy96 + 48);
  fp_set_one(p.z);
  return g1_in_subgroup(p) ? 1 : 0;
}
int ht_g2_in_subgroup(const uint8_t* xy192) {
  g2j p;
  fp_in(p.x.c0, xy192);
  fp_in(p.x.c1, xy192 + 48);
  fp_in(p.y.c0, xy192 + 96);
  fp_in(p.y.c1, xy192 + 144);
  fp2_set_one(p.z);
  return g2_in_subgroup(p) ? 1 : 0;
}
// ops.h g2_subgroup_and_mul_i64: membership and [c] P from one doubling chain (k_tagg_scale's small-integer path)
int ht_g2_subgroup_and_mul_i64(const uint8_t* xy192, int64_t c, uint8_t* out192, int* out_inf) {
  g2j p, q;
  fp_in(p.x.c0, xy192);
  fp_in(p.x.c1, xy192 + 48);
  fp_in(p.y.c0, xy192 + 96);
  fp_in(p.y.c1, xy192 + 144);
  fp2_set_one(p.z);
  const int in = g2_subgroup_and_mul_i64(q, p, c) ? 1 : 0;
  *out_inf = jac_is_inf(q) ? 1 : 0;
  if (!*out_inf) {
    g2a a;
    jac_to_aff(a, q);
    fp_out(out192, a.x.c0);
    fp_out(out192 + 48, a.x.c1);
    fp_out(out192 + 96, a.y.c0);
    fp_out(out192 + 144, a.y.c1);
  }
  return in;
}
void ht_g2_clear_cofactor(const uint8_t* xy192, uint8_t* out192) {
  g2j p, q;
  fp_in(p.x.c0, xy192);
  fp_in(p.x.c1, xy192 + 48);
  fp_in(p.y.c0, xy192 + 96);
  fp_in(p.y.c1, xy192 + 144);
  fp2_set_one(p.z);
  g2_clear_cofactor(q, p);
  g2a a;
  jac_to_aff(a, q);
  fp_out(out192, a.x.c0);
  fp_out(out192 + 48, a.x.c1);
  fp_out(out192 + 96, a.y.c0);
  fp_out(out192 + 144, a.y.c1);
}

// e(P, Q) for affine plain inputs; out = 12 plain Fp coefficients in tower order
// (c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1), each 48 bytes.  Computes f^(3 (p^12-1)/r).
void ht_pairing(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  g1a P[1];
  g2a Q[1];
  bool skip[1] = {false};
  fp_in(P[0].x, p96);
  fp_in(P[0].y, p96 + 48);
  fp_in(Q[0].x.c0, q192);
  fp_in(Q[0].x.c1, q192 + 48);
  fp_in(Q[0].y.c0, q192 + 96);
  fp_in(Q[0].y.c1, q192 + 144);
  fp12 f, e;
  miller_loop_n(f, P, Q, skip, 1);
  final_exponentiation(e, f);
  const fp* c = &e.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, c[i]);
}

// Miller loop only (no final exponentiation), same output layout
void ht_miller(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  g1a P[1];
  g2a Q[1];
  bool skip[1] = {false};
  fp_in(P[0].x, p96);
  fp_in(P[0].y, p96 + 48);
  fp_in(Q[0].x.c0, q192);
  fp_in(Q[0].x.c1, q192 + 48);
  fp_in(Q[0].y.c0, q192 + 96);
  fp_in(Q[0].y.c1, q192 + 144);
  fp12 f;
  miller_loop_n(f, P, Q, skip, 1);
  const fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, c[i]);
}

// The two-pair Miller loop (Verify's shape) with f in registers (lds = 0, pairing.h miller_loop_2) or in the LDS
// layout (lds = 1, pairing_lds.h miller_loop_2_l); out576 = f, outT = the second pair's final T (X, Y, Z: 288 bytes)
void ht_miller2(const uint8_t* p0, const uint8_t* q0, const uint8_t* p1, const uint8_t* q1, int lds,
                uint8_t* out576, uint8_t* outT) {
  g1a P0, P1;
  g2a Q0, Q1;
  fp_in(P0.x, p0);
  fp_in(P0.y, p0 + 48);
  fp_in(P1.x, p1);
  fp_in(P1.y, p1 + 48);
  const uint8_t* qs[2] = {q0, q1};
  g2a* Qs[2] = {&Q0, &Q1};
  for (int k = 0; k < 2; ++k) {
    fp_in(Qs[k]->x.c0, qs[k]);
    fp_in(Qs[k]->x.c1, qs[k] + 48);
    fp_in(Qs[k]->y.c0, qs[k] + 96);
    fp_in(Qs[k]->y.c1, qs[k] + 144);
  }
  fp12 f;
  g2j T;
  if (lds) {
    u32x4 slot[36];
    const f12l<1> F{slot};
    miller_loop_2_l(f, F, P0, Q0, P1, Q1, &T);
  } else {
    miller_loop_2(f, P0, Q0, P1, Q1, &T);
  }
  const fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, c[i]);
  const fp* t = &T.x.c0;
  for (int i = 0; i < 6; ++i) fp_out(outT + 48 * i, t[i]);
}

// Fp12 product / final exponentiation on raw coefficient arrays (plain, tower order)
void ht_final_exp(const uint8_t* in576, uint8_t* out576) {
  fp12 f, e;
  fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_in(c[i], in576 + 48 * i);
  final_exponentiation(e, f);
  const fp* d = &e.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, d[i]);
}

// final_exponentiation_l (pairing_lds.h: the Karabina tail accumulates in the LDS slot), same layout as ht_final_exp
void ht_final_exp_l(const uint8_t* in576, uint8_t* out576) {
  fp12 f, e;
  fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_in(c[i], in576 + 48 * i);
  final_exponentiation_l(e, f, host_f12_slot());
  const fp* d = &e.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, d[i]);
}

void ht_fp12_op(int op, const uint8_t* a576, const uint8_t* b576, uint8_t* out576) {
  fp12 a, b, r;
  fp* ca = &a.c0.c0.c0;
  fp* cb = &b.c0.c0.c0;
  for (int i = 0; i < 12; ++i) {
    fp_in(ca[i], a576 + 48 * i);
    fp_in(cb[i], b576 + 48 * i);
  }
  switch (op) {
    case 0: fp12_mul(r, a, b); break;
    case 1: fp12_sqr(r, a); break;
    case 2: fp12_inv(r, a); break;
    case 3: fp12_frobenius(r, a, 1); break;
    case 4: fp12_frobenius(r, a, 2); break;
    case 5: fp12_frobenius(r, a, 3); break;
    case 6: fp12_cyclotomic_sqr(r, a); break;
    case 7: fp12_mul_line(a, b.c0.c0, b.c0.c1, b.c1.c1); r = a; break;
    case 8: fp12_cyc_exp_xabs_karabina(r, a); break;
    case 9: fp12_cyc_exp_xabs_gs(r, a); break;
    default: r = a;
  }
  const fp* d = &r.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out(out576 + 48 * i, d[i]);
}

int ht_threshold_aggregate(const uint8_t* sigs, const int64_t* ids, int n, uint8_t* out96) {
  return op_threshold_aggregate(out96, sigs, ids, n);  // ops.h: the kernels' two paths (small ids / field)
}

// ops.h lagrange_small: 1 and (c_me, L) when the group takes the small-integer path, else 0.
int ht_lagrange_small(const int64_t* ids, int t, int me, int64_t* c, uint64_t* L) {
  return lagrange_small(ids, t, me, *c, *L) ? 1 : 0;
}

// [k] P on G2 by the 4-dimensional GLS split (k: 8 plain little-endian limbs) or, with glv = 0,
// by plain double-and-add; P is a subgroup-checked compressed point.  Returns the decode status.
int ht_g2_mul(const uint8_t* p96, const uint32_t* k8, int glv, uint8_t* out96) {
  g2a a;
  const int st = g2_decompress(a, p96, true);
  if (st != DEC_OK) return st;
  g2j pj, r;
  jac_from_aff(pj, a);
  if (glv)
    g2_mul_glv4(r, pj, k8);
  else
    jac_mul_limbs(r, pj, k8, 8);
  g2_compress(out96, r);
  return DEC_OK;
}

// Fp-multiplication counts of one op_verify call (mul, sqr)
void ht_count_verify(const uint8_t* pk, const uint8_t* msg, uint32_t len, const uint8_t* sig, uint64_t* out2) {
  g_fp_mul_count = 0;
  g_fp_sqr_count = 0;
  op_verify(pk, msg, len, sig);
  out2[0] = g_fp_mul_count;
  out2[1] = g_fp_sqr_count;
}

// Fp-multiplication counts (mul + sqr) of ONE sigagg group through the stages of hipbls_threshold_aggregate_verify
// (kernels.h): out5[0] every partial's k_tagg_scale work (decode, subgroup test, c_k sig_k or lambda_k sig_k),
// out5[1] k_tagg_sum_s (the sum S, affine), out5[2] k_tagg_unscale ([L^-1] S, compress), out5[3] the key side of
// k_tv_prep_pk (decode + subgroup test, [L] pk, hash_to_G2), out5[4] the pairing check on S against [L] pk (what
// k_verify_pair_lq4 splits over a lane quad).  Returns the verify status.  The C3 roofline unit (bench.py
// TAGG_FPMUL, tests/test_work_counts.py).
int ht_count_tagg_verify(const uint8_t* sigs, const int64_t* ids, int t, const uint8_t* pk48, const uint8_t* msg,
                         uint32_t len, uint64_t* out5) {
  auto take = [](uint64_t* o) {
    *o = g_fp_mul_count + g_fp_sqr_count;
    g_fp_mul_count = 0;
    g_fp_sqr_count = 0;
  };
  if (t < 1 || t > 16) return HIPBLS_ERR_COMBINE;
  g_fp_mul_count = 0;
  g_fp_sqr_count = 0;
  g2j part[16];
  for (int me = 0; me < t; ++me) {  // k_tagg_scale, one lane per partial
    int64_t c = 0;
    uint64_t L = 0;
    const bool small = lagrange_small(ids, t, me, c, L);
    g2a s;
    if (g2_decompress(s, sigs + 96 * me, !small) != DEC_OK) return HIPBLS_ERR_SIGNATURE;
    g2j sj;
    jac_from_aff(sj, s);
    if (small) {
      if (!g2_subgroup_and_mul_i64(part[me], sj, c)) return HIPBLS_ERR_SIGNATURE;
    } else {
      tagg_scale_point(part[me], sj, ids, t, me);
    }
  }
  take(&out5[0]);
  g2j acc;  // k_tagg_sum_s
  jac_set_inf(acc);
  for (int me = 0; me < t; ++me) {
    g2j x = acc;
    jac_add(acc, x, part[me]);
  }
  const bool inf = jac_is_inf(acc);
  g2a S;
  if (!inf) jac_to_aff(S, acc);
  take(&out5[1]);
  g2j u = acc;  // k_tagg_unscale
  if (!inf) jac_from_aff(u, S);
  tagg_unscale(u, ids, t);
  uint8_t sig[96];
  g2_compress(sig, u);
  take(&out5[2]);
  g1a pk;  // k_tv_prep_pk
  if (g1_decompress(pk, pk48, true) != DEC_OK) return HIPBLS_ERR_PUBKEY;
  g1_scale_affine(pk, tagg_group_L(ids, t));
  g2j hj;
  hash_to_g2(hj, msg, len, DST_POP, 43);
  g2a hm;
  jac_to_aff(hm, hj);
  take(&out5[3]);
  const int st = inf ? HIPBLS_ERR_VERIFY : pairing_check_verify_sig(pk, hm, S);  // k_verify_pair_lq4
  take(&out5[4]);
  return st;
}


void ht_reset_counts(void) {
  g_fp_mul_count = 0;
  g_fp_sqr_count = 0;
}
void ht_get_counts(uint64_t* out2) {
  out2[0] = g_fp_mul_count;
  out2[1] = g_fp_sqr_count;
}

}  // extern "C"

// ---- RLC BatchVerify: the four kernel stages of charon_amd/csrc/rlc.h run lane by lane ----------
#include "../../charon_amd/csrc/rlc.h"
#include <vector>

extern "C" int ht_rlc_verify(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                             const uint8_t* msgs, const uint64_t* offs, uint64_t n_msgs, const uint8_t* seed32,
                             int32_t* status, uint64_t* stats3, uint64_t* counts4) {
  // counts4 (optional): Fp products (mul + sqr) spent in each of the four stages
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  std::vector<uint32_t> rpk(n * 36), rsig(n * 72), H((n_msgs ? n_msgs : 1) * 48);
  std::vector<int32_t> win(n_win);
  uint64_t c0 = 0;
  auto mark = [&](int k) {
    const uint64_t c = g_fp_mul_count + g_fp_sqr_count;
    if (counts4) counts4[k] = c - c0;
    c0 = c;
  };
  c0 = g_fp_mul_count + g_fp_sqr_count;
  for (uint64_t i = 0; i < n; ++i) rlc_items_lane(i, pks, sigs, msg_idx, n, n_msgs, seed, rpk.data(), rsig.data(), status);
  mark(0);
  for (uint64_t m = 0; m < n_msgs; ++m) rlc_hash_lane(m, msgs, offs, H.data(), n_msgs, nullptr);
  mark(1);
  std::vector<uint32_t> list;
  for (uint64_t w = 0; w < n_win; ++w)
    if (rlc_window_lane(host_f12_slot(), w, n, msg_idx, rpk.data(), rsig.data(), H.data(), n_msgs, nullptr, status, win.data()))
      for (uint64_t i = w * RLC_W; i < n && i < (w + 1) * RLC_W; ++i)
        if (status[i] == RLC_PENDING) list.push_back((uint32_t)i);
  mark(2);
  for (uint32_t i : list)
    rlc_fallback_lane(host_f12_slot(), i, pks, sigs, msg_idx, H.data(), n_msgs, nullptr, status, nullptr, 0, nullptr,
                      rpk.data(), rsig.data(), n);
  mark(3);
  stats3[0] = n_win;
  stats3[1] = stats3[2] = 0;
  for (int32_t x : win)
    if (x > 0) {
      stats3[1] += 1;
      stats3[2] += (uint64_t)x;
    }
  return 0;
}

// Same pipeline with the public keys from a resident pubshare table (tab_pks, T) by key_idx.
extern "C" int ht_rlc_verify_keys(const uint8_t* tab_pks, uint64_t T, const uint32_t* key_idx, const uint8_t* sigs,
                                  const uint32_t* msg_idx, uint64_t n, const uint8_t* msgs, const uint64_t* offs,
                                  uint64_t n_msgs, const uint8_t* seed32, int32_t* status, int32_t* tab_status,
                                  uint64_t* stats3) {
  std::vector<int32_t> code(T);
  std::vector<uint32_t> tab(T * PUBTAB_WORDS);
  for (uint64_t k = 0; k < T; ++k) tab_status[k] = pubtab_load_lane(k, tab_pks, T, code.data(), tab.data());
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  std::vector<uint32_t> rpk(n * 36), rsig(n * 72), H((n_msgs ? n_msgs : 1) * 48);
  std::vector<int32_t> win(n_win);
  for (uint64_t i = 0; i < n; ++i)
    rlc_items_lane(i, nullptr, sigs, msg_idx, n, n_msgs, seed, rpk.data(), rsig.data(), status, key_idx, T,
                   code.data(), tab.data());
  for (uint64_t m = 0; m < n_msgs; ++m) rlc_hash_lane(m, msgs, offs, H.data(), n_msgs, nullptr);
  std::vector<uint32_t> list;
  for (uint64_t w = 0; w < n_win; ++w)
    if (rlc_window_lane(host_f12_slot(), w, n, msg_idx, rpk.data(), rsig.data(), H.data(), n_msgs, nullptr, status, win.data()))
      for (uint64_t i = w * RLC_W; i < n && i < (w + 1) * RLC_W; ++i)
        if (status[i] == RLC_PENDING) list.push_back((uint32_t)i);
  for (uint32_t i : list)
    rlc_fallback_lane(host_f12_slot(), i, nullptr, sigs, msg_idx, H.data(), n_msgs, nullptr, status, key_idx, T, tab.data(),
                      rpk.data(), rsig.data(), n);
  stats3[0] = n_win;
  stats3[1] = stats3[2] = 0;
  for (int32_t x : win)
    if (x > 0) {
      stats3[1] += 1;
      stats3[2] += (uint64_t)x;
    }
  return 0;
}

// tbls.Verify with the key from a table (k_verify_keys body)
extern "C" int ht_verify_key(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* sig) {
  int32_t code;
  uint32_t tab[PUBTAB_WORDS];
  pubtab_load_lane(0, pk48, 1, &code, tab);
  g1a pk;
  g1j xpk;
  const int dp = pubtab_get(pk, xpk, 0, 1, &code, tab);
  return op_verify_decoded_pk(dp, pk, msg, len, sig, host_f12_slot());
}

// ---- batch-wide RLC check with the Pippenger MSM (charon_amd/csrc/rlcb.h), lane by lane ------------------
#include "../../charon_amd/csrc/rlcb.h"

namespace {
// Pippenger over npts affine AoS points (rlcb.h layout) with 32-bit scalars: the device stages run serially; W = the window sums.
void host_msm(g2j* W, const uint32_t* pts, const uint32_t* sc, uint64_t npts) {
  std::vector<uint32_t> cnt(MSM_WINDOWS * MSM_NB, 0), off(MSM_WINDOWS * (MSM_NB + 1)), cur(MSM_WINDOWS * MSM_NB);
  std::vector<uint32_t> list(MSM_WINDOWS * (npts ? npts : 1));
  for (uint64_t p = 0; p < npts; ++p) msm_hist_lane(p, sc, cnt.data());
  for (int w = 0; w < MSM_WINDOWS; ++w) {
    uint32_t acc = 0;
    for (uint32_t j = 0; j < MSM_NB; ++j) {
      off[w * (MSM_NB + 1) + j] = acc;
      cur[w * MSM_NB + j] = acc;
      acc += cnt[w * MSM_NB + j];
    }
    off[w * (MSM_NB + 1) + MSM_NB] = acc;
  }
  for (uint64_t p = 0; p < npts; ++p) msm_scatter_lane(p, sc, cur.data(), list.data(), npts);
  const uint64_t lpw = msm_run_lanes(npts);
  std::vector<uint32_t> B((uint64_t)MSM_WINDOWS * MSM_NB * 72), Sg((uint64_t)MSM_WINDOWS * MSM_NSEG * 72);
  std::vector<uint32_t> P(2 * MSM_WINDOWS * (lpw ? lpw : 1) * 72);
  for (int w = 0; w < MSM_WINDOWS; ++w)
    for (uint64_t r = 0; r < lpw; ++r) msm_run_lane(w, r, off.data(), list.data(), npts, pts, B.data(), P.data(), lpw);
  for (int w = 0; w < MSM_WINDOWS; ++w)
    for (uint32_t j = 0; j < MSM_NB; ++j) msm_fix_lane(w, j, off.data(), B.data(), P.data(), lpw);
  for (int w = 0; w < MSM_WINDOWS; ++w)
    for (uint32_t s = 0; s < MSM_NSEG; ++s) msm_segment_lane(w, s, B.data(), Sg.data());
  for (int w = 0; w < MSM_WINDOWS; ++w) {
    jac_set_inf(W[w]);
    for (uint32_t s = 0; s < MSM_NSEG; ++s) {
      g2j t;
      soa_load<72>(&t.x.c0.v[0], Sg.data(), (uint64_t)MSM_WINDOWS * MSM_NSEG, (uint64_t)w * MSM_NSEG + s);
      jac_add(W[w], W[w], t);
    }
  }
}
}  // namespace

// sum_i [sc_i] P_i for affine plain points (x0, x1, y0, y1 big-endian, 192 B each); out = compressed 96 B
extern "C" void ht_msm_g2(const uint8_t* pts192, const uint32_t* sc, uint64_t n, uint8_t* out96) {
  std::vector<uint32_t> pts(48 * (n ? n : 1));
  for (uint64_t i = 0; i < n; ++i) {
    g2a a;
    fp_in(a.x.c0, pts192 + 192 * i);
    fp_in(a.x.c1, pts192 + 192 * i + 48);
    fp_in(a.y.c0, pts192 + 192 * i + 96);
    fp_in(a.y.c1, pts192 + 192 * i + 144);
    aos_store<48>(pts.data(), i, &a.x.c0.v[0]);
  }
  g2j W[MSM_WINDOWS], S;
  host_msm(W, pts.data(), sc, n);
  msm_combine(S, W[0], W[1]);
  g2_compress(out96, S);
}

// The batch-check pipeline (stages 1-6 of rlcb.h) followed by the window/fallback stages of rlc.h for whatever
// the batch check left pending.  *passed = the batch-wide verdict.
// counts6 (optional): Fp products of items, hash, MSM, chunk Miller loops, product + verdict, windows + fallback.
extern "C" int ht_rlcb_verify(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                              const uint8_t* msgs, const uint64_t* offs, uint64_t n_msgs, const uint8_t* seed32,
                              int32_t* status, int32_t* passed, uint64_t* counts6) {
  uint64_t c0 = g_fp_mul_count + g_fp_sqr_count;
  auto mark = [&](int k) {
    const uint64_t c = g_fp_mul_count + g_fp_sqr_count;
    if (counts6) counts6[k] = c - c0;
    c0 = c;
  };
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  std::vector<uint32_t> rpk(n * 36), rsig(n * 72), pts(2 * n * 48), sc(2 * n), H((n_msgs ? n_msgs : 1) * 48);
  // the G1 MSM per large message (g1msm.h) under the runtime's rule (hipbls.hip launch_rlc_batch)
  const uint32_t g1min = g_g1m_min;
  const bool g1 = g1min > 0 && n_msgs > 0 && n >= 8 * n_msgs && n >= g1min;
  const uint64_t nl_max = g1 ? std::min<uint64_t>(n_msgs, n / g1min) : 0;
  std::vector<uint32_t> gcnt(n_msgs + 1, 0), lid(n_msgs + 1), lmsg(nl_max + 1), soff(nl_max + 2), gcur(nl_max + 1, 0);
  std::vector<uint32_t> meta(2, 0), pos(n + 1), slotl(n + 1), gpts(60 * n + 4), gsc(2 * n + 2);
  if (g1) {
    for (uint64_t i = 0; i < n; ++i)
      if (msg_idx[i] < n_msgs) gcnt[msg_idx[i]] += 1;
    g1m_plan_serial(gcnt.data(), n_msgs, g1min, lid.data(), lmsg.data(), soff.data(), meta.data());
    for (uint64_t i = 0; i < n; ++i)
      g1m_rank_lane(i, msg_idx, n_msgs, lid.data(), soff.data(), gcur.data(), pos.data(), slotl.data());
  }
  const uint32_t* gpos = g1 ? pos.data() : nullptr;
  for (uint64_t i = 0; i < n; ++i)
    rlcb_items_lane(i, pks, sigs, msg_idx, n, n_msgs, seed, rpk.data(), pts.data(), sc.data(), status, nullptr, 0,
                    nullptr, nullptr, gpos, gpts.data(), gsc.data());
  mark(0);
  for (uint64_t m = 0; m < n_msgs; ++m) rlc_hash_lane(m, msgs, offs, H.data(), n_msgs, nullptr);
  mark(1);
  g2j W[MSM_WINDOWS];
  host_msm(W, pts.data(), sc.data(), 2 * n);
  std::vector<uint32_t> Wc(2 * 72);
  for (int k = 0; k < 72; ++k) {
    Wc[k] = (&W[0].x.c0.v[0])[k];
    Wc[72 + k] = (&W[1].x.c0.v[0])[k];
  }
  const uint64_t nb = nl_max * G1M_NBL;
  std::vector<uint32_t> bcnt(nb + 1, 0), boff(nb + 1), bcur(nb + 1), glist(2 * G1M_WIN * n + 1), B(36 * nb + 4);
  std::vector<uint32_t> Wv(36 * nl_max * G1M_NFOLD + 4);
  if (g1) {  // counted with the MSM (stage 2 of counts6)
    for (uint64_t t = 0; t < n; ++t) g1m_hist_lane(t, meta.data(), gsc.data(), slotl.data(), bcnt.data());
    uint32_t acc = 0;
    for (uint64_t b = 0; b < nb; ++b) {
      boff[b] = bcur[b] = acc;
      acc += bcnt[b];
    }
    boff[nb] = acc;
    for (uint64_t t = 0; t < n; ++t) g1m_scatter_lane(t, meta.data(), gsc.data(), slotl.data(), bcur.data(), glist.data());
    const uint64_t nrun = g1m_run_lanes(n);
    std::vector<uint32_t> P(2 * 36 * nrun + 4);
    for (uint64_t r = 0; r < nrun; ++r) g1m_run_lane(r, meta.data(), boff.data(), glist.data(), gpts.data(), n, B.data(), P.data());
    for (uint64_t b = 0; b < nb; ++b) g1m_fix_lane(b, meta.data(), boff.data(), B.data(), P.data());
    for (uint64_t q = 0; q < nl_max * G1M_NFOLD; ++q) g1m_fold_lane(q, meta.data(), B.data(), Wv.data());
  }
  mark(2);
  // stage 3 as the device runs it: the chunks, then the (-g1, S) lane as the last column
  // (then the large messages' Miller values, as the device's k_g1m_miller columns)
  const uint64_t nch = g_rlcb_chunks ? g_rlcb_chunks : rlcb_chunk_count(n, g_rlcb_slots);
  const uint64_t cols = nch + 1 + nl_max;
  std::vector<uint32_t> F(144 * cols);
  for (uint64_t c = 0; c < nch; ++c)
    rlcb_chunk_lane(host_f12_slot(), c, n, status, msg_idx, rpk.data(), H.data(), n_msgs, nullptr, F.data(), nch,
                    cols);
  for (uint64_t L = 0; L < nl_max; ++L)
    g1m_miller_lane(host_f12_slot(), L, meta.data(), lmsg.data(), Wv.data(), H.data(), n_msgs, nullptr, F.data(),
                    nch + 1 + L, cols);
  mark(3);  // the (-g1, S) lane is counted with the product and the verdict (stage 4 of counts6)
  rlcb_sfactor_lane(host_f12_slot(), Wc.data(), F.data(), cols, nch);
  uint64_t cur = cols;
  while (cur > 1) {
    const uint64_t nxt = (cur + RLCB_FAN - 1) / RLCB_FAN;
    std::vector<uint32_t> G(144 * nxt);
    for (uint64_t g = 0; g < nxt; ++g) fp12_prod_lane(g, F.data(), cur, G.data(), nxt, RLCB_FAN);
    F.swap(G);
    cur = nxt;
  }
  bool any = false;
  for (uint64_t i = 0; i < n; ++i) any = any || status[i] == RLC_PENDING;
  bool pass = true;
  if (any) {
    fp12 f;
    soa_load<144>(&f.c0.c0.c0.v[0], F.data(), 1, 0);
    fp12 e;
    final_exponentiation(e, f);
    pass = fp12_is_one(e);
  }
  for (uint64_t i = 0; i < n; ++i)
    rlcb_mark_lane(i, n, pass, status, pts.data(), sc.data(), rsig.data(), gpos, gpts.data(), gsc.data(), rpk.data());
  *passed = pass ? 1 : 0;
  mark(4);
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  std::vector<int32_t> win(n_win ? n_win : 1);
  std::vector<uint32_t> list;
  for (uint64_t w = 0; w < n_win; ++w)
    if (rlc_window_lane(host_f12_slot(), w, n, msg_idx, rpk.data(), rsig.data(), H.data(), n_msgs, nullptr, status, win.data()))
      for (uint64_t i = w * RLC_W; i < n && i < (w + 1) * RLC_W; ++i)
        if (status[i] == RLC_PENDING) list.push_back((uint32_t)i);
  for (uint32_t i : list)
    rlc_fallback_lane(host_f12_slot(), i, pks, sigs, msg_idx, H.data(), n_msgs, nullptr, status, nullptr, 0, nullptr,
                      rpk.data(), rsig.data(), n);
  mark(5);
  return 0;
}

// ---- binary-GCD inversion (field.h fp_inv) against the Fermat power, on plain-limb inputs ------------------
// one fp_mul on raw little-endian limbs (no range check of its own: tests/test_operand_contract.py)
extern "C" void ht_fp_mul_raw(const uint32_t* a12, const uint32_t* b12, uint32_t* out12) {
  fp a, b, r;
  for (int i = 0; i < 12; ++i) {
    a.v[i] = a12[i];
    b.v[i] = b12[i];
  }
  fp_mul(r, a, b);
  for (int i = 0; i < 12; ++i) out12[i] = r.v[i];
}

extern "C" void ht_fp_inv(const uint32_t* x12, int gcd, uint32_t* out12) {
  fp x, r;
  for (int i = 0; i < 12; ++i) x.v[i] = x12[i];
  if (gcd)
    fp_inv(r, x);
  else
    fp_inv_pow(r, x);
  for (int i = 0; i < 12; ++i) out12[i] = r.v[i];
}

extern "C" void ht_rlcb_set_slots(uint64_t slots) { g_rlcb_slots = slots; }
extern "C" void ht_rlcb_set_chunks(uint64_t nch) { g_rlcb_chunks = nch; }
extern "C" uint32_t ht_rlcb_set_g1_min(uint32_t min) {
  const uint32_t o = g_g1m_min;
  g_g1m_min = min;
  return o;
}
extern "C" uint64_t ht_rlcb_chunk_count(uint64_t n, uint64_t slots) { return rlcb_chunk_count(n, slots); }
