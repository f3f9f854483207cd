// Batch-wide RLC check with a Pippenger MSM (BASELINE.json north star: "Random-linear-combination batch
// verification uses a Pippenger MSM over G1/G2 with LDS-staged bucket accumulation").
//
// The windowed RLC of rlc.h gives every window of 8 items its own final exponentiation, because at the bench's
// 1 % invalid partials a single batch-wide check fails on every batch.  When invalid partials are rare (the
// normal case for a healthy cluster), one check over the whole batch is much cheaper:
//
//     prod_runs e( sum_{i in run} r_i pk_i , H(m_run) ) * e( -g1 , sum_i r_i sig_i ) == 1
//
// with the same per-item scalars r_i = a_i + b_i x as the windows (rlc_scalars), so the windows can take over
// without recomputing anything when the batch check fails.  Stages (one lane per unit; kernels.h, hipbls.hip):
//   1. items    : decode + subgroup tests (herumi's order, final statuses), [r_i] pk_i in G1 (Shamir, as rlc.h),
//                 and the MSM inputs sig_i, psi(sig_i) (affine, psi = [x] on G2) with 32-bit scalars a_i, b_i;
//   2. MSM      : S = sum_i [a_i] sig_i + [b_i] psi(sig_i), Pippenger with 16-bit windows: counting sort of the
//                 2n points by digit (histogram, scan, scatter), one lane per bucket sums its points, one lane
//                 per 16-bucket segment folds sum_j j B_j by running sums, two workgroups tree-sum the
//                 segments in LDS, and S = W0 + [2^16] W1;
//   3. chunks   : one lane per ~16 consecutive items: runs of equal message among pending items are summed in G1
//                 and paired with H(m) in one multi-Miller loop (no final exponentiation) -> f_chunk; beside them
//                 the S factor: S from the window sums and the Miller value of (-g1, S) (rlcb_sfactor_lane; on the
//                 device a split-Fp2 lane group, verify_lat.hip k_rlcb_sfactor8); committee roots add one Miller
//                 value per large message (g1msm.h);
//   4. product  : the Miller values multiplied together (host: fan-in RLCB_FAN per level; device: 64 per wave,
//                 kernels.h k_fp12_prod64);
//   5. final    : the product times the S factor and the final exponentiation (device: a lane quad with Fp2
//                 twins, verify_lat.hip k_rlcb_final8); the verdict goes to a device flag;
//   6. mark     : pass -> every pending item is valid; fail -> each pending item gets [r_i] sig_i for the window
//                 stages of rlc.h, which then decide item by item.
// Soundness is the windows' argument over the whole batch: a batch with an invalid item passes with
// probability <= 2^-64 over the scalars.  Bucket 0 is skipped (digit 0 adds nothing).
#pragma once
#include "rlc.h"

namespace bls {

constexpr int RLCB_C = 16;                     // items per Miller chunk (target)
constexpr int RLCB_CMAX = 18;                  // most items a chunk lane may get (rlcb_chunk_count)
constexpr int MSM_BITS = 16;                   // Pippenger window width
constexpr int MSM_WINDOWS = 2;                 // 32-bit scalars
constexpr uint32_t MSM_NB = 1u << MSM_BITS;    // buckets per window (bucket 0 unused)
constexpr int MSM_SEG = 8;                     // buckets folded per segment lane
constexpr uint32_t MSM_NSEG = MSM_NB / MSM_SEG;
constexpr int MSM_RUN = 64;                    // bucket-sorted list entries per bucket-run lane
constexpr int MSM_WG = 8;                      // workgroups folding one window's segment results
// Fan-in of the Miller-value product tree: a level costs `fan` serial Fp12 products, so f * log_f(chunks) products
// of latency in all -- 32 at fan 4 for 65,536 chunks, 64 at fan 16.
constexpr int RLCB_FAN = 4;

#if defined(__HIP_DEVICE_COMPILE__)
#define BLS_ATOMIC_ADD_U32(p, v) atomicAdd((p), (v))
#else
BLS_HD BLS_INLINE uint32_t bls_serial_add_u32(uint32_t* p, uint32_t v) {  // host build: lanes run one by one
  const uint32_t o = *p;
  *p = o + v;
  return o;
}
#define BLS_ATOMIC_ADD_U32(p, v) bls_serial_add_u32((p), (v))
#endif
}  // namespace bls
#include "g1msm.h"
namespace bls {

// ---- stage 1 ------------------------------------------------------------------------------------
// pts: 2n affine G2 points, point-major (AoS, 48 contiguous words each: sig_i at i, psi(sig_i) at n + i), because
// the bucket stage gathers them by index -- limb-major SoA made every gathered point 48 separate cache lines
// (profiles/r04: k_msm_bucket moved 23 GB per launch for 0.8 GB of points); sc: 2n scalars (a_i, then b_i).
BLS_HD BLS_INLINE void rlcb_items_lane(uint64_t i, const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx,
                                       uint64_t n, uint64_t n_msgs, const rlc_seed& seed, uint32_t* rpk,
                                       uint32_t* pts, uint32_t* sc, int32_t* status,
                                       const uint32_t* key_idx = nullptr, uint64_t T = 0,
                                       const int32_t* tcode = nullptr, const uint32_t* tab = nullptr,
                                       const uint32_t* g1pos = nullptr, uint32_t* gpts = nullptr,
                                       uint32_t* gsc = nullptr) {
  g1j rp;
  jac_set_inf(rp);
  g2a sig, psig;
  fp2_set_zero(sig.x);
  fp2_set_zero(sig.y);
  psig = sig;
  uint32_t a = 0, b = 0;
  int st;
  if (msg_idx[i] >= n_msgs || (!pks && key_idx[i] >= T)) {
    st = HIPBLS_ERR_ARG;
  } else {
    // items of a message with many items (g1msm.h): [r] pk comes from the message's G1 MSM, not from this lane
    const uint32_t slot = g1pos ? g1pos[i] : G1M_NONE;
    g1a pk;
    g1j xpk;
    const int dp = pks ? g1_decompress_keep_x(pk, xpk, pks + 48 * i) : pubtab_get(pk, xpk, key_idx[i], T, tcode, tab);
    st = RLC_PENDING;
    if (dp == DEC_BAD) st = HIPBLS_ERR_PUBKEY;
    if (st == RLC_PENDING) {
      const int ds = g2_decompress(sig, sigs + 96 * i, true);
      if (ds == DEC_BAD)
        st = HIPBLS_ERR_SIGNATURE;
      else if (dp == DEC_INF || ds == DEC_INF)
        st = HIPBLS_ERR_VERIFY;
    }
    if (st == RLC_PENDING) {
      rlc_scalars(a, b, seed, i);
      if (slot == G1M_NONE) {
        g1j pj;
        jac_from_aff(pj, pk);
        jac_mul2_u32(rp, pj, xpk, a, b);
      }
      g2j sj, psj;
      jac_from_aff(sj, sig);
      g2_psi(psj, sj);  // Z stays 1: psi of an affine point is affine
      psig.x = psj.x;
      psig.y = psj.y;
    } else {
      fp2_set_zero(sig.x);
      fp2_set_zero(sig.y);
    }
    if (slot != G1M_NONE) g1m_store_slot(gpts, gsc, n, slot, st == RLC_PENDING, pk, xpk, a, b);
  }
  soa_store<36>(rpk, n, i, &rp.x.v[0]);
  aos_store<48>(pts, i, &sig.x.c0.v[0]);
  aos_store<48>(pts, n + i, &psig.x.c0.v[0]);
  sc[i] = a;
  sc[n + i] = b;
  status[i] = st;
}

// ---- stage 2: Pippenger ----------------------------------------------------------------------------
BLS_HD BLS_INLINE uint32_t msm_digit(uint32_t s, int w) { return (s >> (MSM_BITS * w)) & (MSM_NB - 1); }

// cnt: MSM_WINDOWS x MSM_NB counters (zeroed)
BLS_HD BLS_INLINE void msm_hist_lane(uint64_t p, const uint32_t* sc, uint32_t* cnt) {
  const uint32_t s = sc[p];
  for (int w = 0; w < MSM_WINDOWS; ++w) {
    const uint32_t d = msm_digit(s, w);
    if (d) BLS_ATOMIC_ADD_U32(&cnt[w * MSM_NB + d], 1u);
  }
}

// cursor: the exclusive scan of cnt (per window); list: MSM_WINDOWS x npts point indices grouped by bucket
BLS_HD BLS_INLINE void msm_scatter_lane(uint64_t p, const uint32_t* sc, uint32_t* cursor, uint32_t* list,
                                        uint64_t npts) {
  const uint32_t s = sc[p];
  for (int w = 0; w < MSM_WINDOWS; ++w) {
    const uint32_t d = msm_digit(s, w);
    if (d) {
      const uint32_t at = BLS_ATOMIC_ADD_U32(&cursor[w * MSM_NB + d], 1u);
      list[(uint64_t)w * npts + at] = (uint32_t)p;
    }
  }
}

// Bucket sums, load-balanced: bucket-run lane r of window w adds the MSM_RUN consecutive entries [r RUN, (r + 1) RUN)
// of the window's bucket-sorted list, whatever buckets they belong to, so every lane does the same number of mixed
// additions (one lane per bucket made each wave as long as its largest bucket: Poisson(32) sizes, ~1.7x the mean).
// A bucket whose entries all lie in the lane's range is written to B directly; a bucket cut by the range's start or
// end leaves a partial sum in P (slot 0 = the lane's first run, slot 1 = its last), which msm_fix_lane adds up.
// off: MSM_WINDOWS x (MSM_NB + 1) exclusive offsets.  B: Jacobian SoA, 72 words x (MSM_WINDOWS * MSM_NB).  P: Jacobian
// SoA, 72 words x (2 * MSM_WINDOWS * lpw), lpw = msm_run_lanes(npts) lanes per window.  Software-pipelined: the next
// point's gather is issued before the current addition; the addition is inlined (jac_add_aff_body), so the
// accumulator and the prefetched point stay in registers.
BLS_HD BLS_INLINE uint64_t msm_run_lanes(uint64_t npts) { return (npts + MSM_RUN - 1) / MSM_RUN; }

BLS_HD BLS_INLINE void msm_run_lane(uint32_t w, uint64_t r, const uint32_t* off, const uint32_t* list, uint64_t npts,
                                    const uint32_t* pts, uint32_t* B, uint32_t* P, uint64_t lpw) {
  const uint32_t* o = off + (uint64_t)w * (MSM_NB + 1);
  const uint64_t total = o[MSM_NB];
  const uint64_t k0 = r * MSM_RUN;
  if (k0 >= total) return;
  const uint64_t k1 = k0 + MSM_RUN < total ? k0 + MSM_RUN : total;
  uint32_t lo = 0, hi = MSM_NB;  // the bucket of entry k0: o[lo] <= k0 < o[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (o[mid] <= k0)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t j = lo;
  uint64_t end = o[j + 1];
  const uint64_t lane = (uint64_t)w * lpw + r, nb = (uint64_t)MSM_WINDOWS * MSM_NB, ps = 2 * MSM_WINDOWS * lpw;
  const uint32_t* lw = list + (uint64_t)w * npts;
  int slot = 0;
  g2j acc;
  jac_set_inf(acc);
  g2a q;
  aos_load<48>(&q.x.c0.v[0], pts, lw[k0]);
  for (uint64_t k = k0; k < k1; ++k) {
    const g2a cur = q;
    if (k + 1 < k1) aos_load<48>(&q.x.c0.v[0], pts, lw[k + 1]);
    g2j x = acc, y;
    jac_add_aff_body(y, x, cur);
    acc = y;
    if (k + 1 == end || k + 1 == k1) {  // bucket j's run in this range ends here
      if (o[j] >= k0 && end <= k1)
        soa_store<72>(B, nb, (uint64_t)w * MSM_NB + j, &acc.x.c0.v[0]);
      else
        soa_store<72>(P, ps, 2 * lane + slot, &acc.x.c0.v[0]);
      slot = 1;
      jac_set_inf(acc);
      if (k + 1 < k1) {
        ++j;
        while (o[j + 1] <= k + 1) ++j;  // the next non-empty bucket
        end = o[j + 1];
      }
    }
  }
}

// Bucket (w, j) after the run lanes: infinity when empty; written already when its entries fall in one run lane's
// range; otherwise the sum of its partials -- slot 0 of every lane whose range starts inside the bucket, and the first
// lane's slot 0 or 1 depending on whether the bucket starts that lane's range.
BLS_HD BLS_INLINE void msm_fix_lane(uint32_t w, uint32_t j, const uint32_t* off, uint32_t* B, const uint32_t* P,
                                    uint64_t lpw) {
  const uint32_t* o = off + (uint64_t)w * (MSM_NB + 1);
  const uint64_t k0 = o[j], k1 = o[j + 1], nb = (uint64_t)MSM_WINDOWS * MSM_NB, ps = 2 * MSM_WINDOWS * lpw;
  g2j acc;
  if (k0 == k1) {
    jac_set_inf(acc);
    soa_store<72>(B, nb, (uint64_t)w * MSM_NB + j, &acc.x.c0.v[0]);
    return;
  }
  const uint64_t a = k0 / MSM_RUN, b = (k1 - 1) / MSM_RUN;
  if (a == b) return;
  const uint64_t base = 2 * ((uint64_t)w * lpw);
  soa_load<72>(&acc.x.c0.v[0], P, ps, base + 2 * a + (k0 == a * MSM_RUN ? 0 : 1));
  for (uint64_t l = a + 1; l <= b; ++l) {
    g2j p, x = acc, y;
    soa_load<72>(&p.x.c0.v[0], P, ps, base + 2 * l);
    jac_add_body(y, x, p);
    acc = y;
  }
  soa_store<72>(B, nb, (uint64_t)w * MSM_NB + j, &acc.x.c0.v[0]);
}

// segment (w, s): sum_{j in [16 s, 16 s + 16)} j B_j = T + (16 s - 1) R with R = sum B_j and T = sum (j - 16 s + 1) B_j
// from running sums (top bucket first).  Sg: Jacobian SoA, 72 words x (MSM_WINDOWS * MSM_NSEG).  The next bucket is
// loaded before the current one's two additions (as msm_run_lane).
BLS_HD BLS_INLINE void msm_segment_lane(uint32_t w, uint32_t s, const uint32_t* B, uint32_t* Sg) {
  g2j R, T;
  jac_set_inf(R);
  jac_set_inf(T);
  const uint64_t nb = (uint64_t)MSM_WINDOWS * MSM_NB, base = (uint64_t)w * MSM_NB + s * MSM_SEG;
  g2j b;
  soa_load<72>(&b.x.c0.v[0], B, nb, base + MSM_SEG - 1);
  for (int k = MSM_SEG - 1; k >= 0; --k) {
    const g2j cur = b;
    if (k > 0) soa_load<72>(&b.x.c0.v[0], B, nb, base + k - 1);
    g2j x = R, y;
    jac_add_body(y, x, cur);
    R = y;
    g2j u = T, v;
    jac_add_body(v, u, R);
    T = v;
  }
  g2j m, out;
  if (s == 0) {
    jac_neg(m, R);
  } else {
    jac_mul_u64(m, R, (uint64_t)s * MSM_SEG - 1);
  }
  jac_add(out, T, m);
  soa_store<72>(Sg, (uint64_t)MSM_WINDOWS * MSM_NSEG, (uint64_t)w * MSM_NSEG + s, &out.x.c0.v[0]);
}

// S = W0 + [2^16] W1
BLS_HD BLS_INLINE void msm_combine(g2j& S, const g2j& W0, const g2j& W1) {
  g2j t = W1;
  for (int k = 0; k < MSM_BITS; ++k) {
    g2j u;
    jac_dbl(u, t);
    t = u;
  }
  jac_add(S, W0, t);
}

// ---- stage 3: per-chunk multi-Miller loop ----------------------------------------------------------
// How many chunks for n items: ceil(n / RLCB_C), unless that fills whole rounds of waves exactly (`slots` = the waves
// the device runs at once at one wave per SIMD): then one wave fewer, items spread over the lanes (16 or 17 each), so
// a SIMD stays free for the (-g1, S) Miller value beside the chunks (verify_lat.hip k_rlcb_sfactor8).  At the bench's 1M items:
// 65,536 chunks = 1,024 waves = every SIMD, so 65,472.
BLS_HD BLS_INLINE uint64_t rlcb_chunk_count(uint64_t n, uint64_t slots) {
  const uint64_t nch = (n + RLCB_C - 1) / RLCB_C;
  const uint64_t waves = (nch + 63) / 64;
  if (slots == 0 || waves <= 1 || waves < slots || waves % slots != 0) return nch;
  const uint64_t fewer = (waves - 1) * 64;
  return (n + fewer - 1) / fewer <= (uint64_t)RLCB_CMAX ? fewer : nch;
}

// F: Fp12 SoA, 144 words x n_chunks.  Chunk c covers items [c n / n_chunks, (c + 1) n / n_chunks) (at most RLCB_CMAX).
// Chunks without pending items store 1.
template <int S>
BLS_HD BLS_INLINE void rlcb_chunk_lane(const f12l<S>& Lf, uint64_t c, uint64_t n, const int32_t* status, const uint32_t* msg_idx,
                                       const uint32_t* rpk, const uint32_t* H, uint64_t hstride,
                                       const uint32_t* hslot, uint32_t* F, uint64_t n_chunks, uint64_t fstride) {
  g1a P[RLCB_CMAX];
  g2a Q[RLCB_CMAX];
  int np = 0;
  g1j run;
  jac_set_inf(run);
  uint32_t run_msg = 0xffffffffu;
  const uint64_t i0 = c * n / n_chunks, i1 = (c + 1) * n / n_chunks;
  for (uint64_t i = i0; i < i1; ++i) {
    if (status[i] != RLC_PENDING) continue;
    g1j qp;
    soa_load<36>(&qp.x.v[0], rpk, n, i);
    const uint32_t m = msg_idx[i];
    if (m != run_msg) {
      if (run_msg != 0xffffffffu && !jac_is_inf(run)) {
        jac_to_aff(P[np], run);
        soa_load<48>(&Q[np].x.c0.v[0], H, hstride, h_col(hslot, run_msg));
        ++np;
      }
      run = qp;
      run_msg = m;
    } else {
      g1j x = run, y;
      jac_add(y, x, qp);
      run = y;
    }
  }
  if (run_msg != 0xffffffffu && !jac_is_inf(run)) {
    jac_to_aff(P[np], run);
    soa_load<48>(&Q[np].x.c0.v[0], H, hstride, h_col(hslot, run_msg));
    ++np;
  }
  fp12 f;
  if (np)
    miller_loop_multi_l<RLCB_CMAX>(f, Lf, P, Q, np);
  else
    fp12_set_one(f);
  soa_store<144>(F, fstride, c, &f.c0.c0.c0.v[0]);
}

// The S lane of stage 3: S = W0 + [2^16] W1 from the window sums (W: 2 x 72 words, contiguous), then the Miller
// value of (-g1, S) (1 when S is the point at infinity) into column `col` of F.
template <int LS>
BLS_HD BLS_INLINE void rlcb_sfactor_lane(const f12l<LS>& Lf, const uint32_t* W, uint32_t* F, uint64_t stride, uint64_t col) {
  g2j W0, W1, S;
  for (int k = 0; k < 72; ++k) {
    (&W0.x.c0.v[0])[k] = W[k];
    (&W1.x.c0.v[0])[k] = W[72 + k];
  }
  msm_combine(S, W0, W1);
  fp12 f;
  if (jac_is_inf(S)) {
    fp12_set_one(f);
  } else {
    g1a P[1];
    g2a Q[1];
    P[0].x = G1_GEN_X;
    P[0].y = G1_NEG_GEN_Y;
    jac_to_aff(Q[0], S);
    miller_loop_multi_l<1>(f, Lf, P, Q, 1);
  }
  soa_store<144>(F, stride, col, &f.c0.c0.c0.v[0]);
}

// ---- stage 4: product of Miller values, fan-in `fan` ----------------------------------------------------
BLS_HD BLS_INLINE void fp12_prod_lane(uint64_t g, const uint32_t* Fin, uint64_t nin, uint32_t* Fout, uint64_t nout,
                                      int fan) {
  fp12 acc;
  fp12_set_one(acc);
  const uint64_t k0 = g * (uint64_t)fan, k1 = k0 + fan < nin ? k0 + fan : nin;
  for (uint64_t k = k0; k < k1; ++k) {
    fp12 f;
    soa_load<144>(&f.c0.c0.c0.v[0], Fin, nin, k);
    fp12 x = acc, y;
    fp12_mul(y, x, f);
    acc = y;
  }
  soa_store<144>(Fout, nout, g, &acc.c0.c0.c0.v[0]);
}

// ---- stage 6 -------------------------------------------------------------------------------------
// pass: every pending item is valid.  Otherwise [r_i] sig_i = [a_i] sig_i + [b_i] psi(sig_i) goes to rsig (Jacobian
// SoA, 72 x n) for the window stages, which decide the pending items.
BLS_HD BLS_INLINE void rlcb_mark_lane(uint64_t i, uint64_t n, bool pass, int32_t* status, const uint32_t* pts,
                                      const uint32_t* sc, uint32_t* rsig, const uint32_t* g1pos = nullptr,
                                      const uint32_t* gpts = nullptr, const uint32_t* gsc = nullptr,
                                      uint32_t* rpk = nullptr) {
  if (status[i] != RLC_PENDING) return;
  if (pass) {
    status[i] = HIPBLS_OK;
    return;
  }
  if (g1pos && g1pos[i] != G1M_NONE) {  // stage 1 left [r] pk to the G1 MSM: the windows need it per item
    g1j rp;
    g1m_item_rpk(rp, gpts, n, gsc, g1pos[i]);
    soa_store<36>(rpk, n, i, &rp.x.v[0]);
  }
  g2a s, ps;
  aos_load<48>(&s.x.c0.v[0], pts, i);
  aos_load<48>(&ps.x.c0.v[0], pts, n + i);
  g2j rs;
  jac_mul2_u32_aff(rs, s, ps, sc[i], sc[n + i]);
  soa_store<72>(rsig, n, i, &rs.x.c0.v[0]);
}

}  // namespace bls
