// The G1 half of the batch-wide RLC check's Pippenger MSM (BASELINE.json north star: "a Pippenger MSM over G1/G2"):
// for every message with many items -- committee roots, where one signing root is shared by a whole committee's
// partials (/root/reference/core/validatorapi/validatorapi.go:246-283, grouped by root in core/parsigdb/memory.go:
// 198-225) -- one bucket-method sum
//     R_m = sum_{i : msg i = m} [r_i] pk_i = sum_i [a_i] pk_i + [b_i] ([x] pk_i)          (r_i = a_i + b_i x, rlc.h)
// replaces the per-item Shamir multiplication [r_i] pk_i of rlcb.h stage 1, and ONE Miller pair (R_m, H(m)) per such
// message replaces its share of the chunk Miller loops.  The other messages keep the per-item path; the verdict and
// every status are unchanged (the batch equation is the same group element either way).
//
// Layout (one "large" message L = its dense index among messages with >= min items):
//   * slots: the large messages' items, message by message (soff[L] .. soff[L + 1]); slot s holds pk_s affine
//     (24 words at gpts + 24 s) and [x] pk_s Jacobian as the subgroup check left it (36 words at gxp + 36 s, gxp =
//     gpts + 24 n: no inversion per item), both point-major so the bucket lanes gather them by index, and the
//     scalars (a_s, b_s); an item that did not decode keeps zero scalars and adds nothing;
//   * buckets: per (L, kind, window w of 4 bits, digit d = 1..15), kind 0 = pk with a's digits (mixed additions),
//     kind 1 = [x] pk with b's digits (full additions); each kind has 128 bucket indices of which 120 are used, so a
//     wave of bucket lanes never mixes the two addition formulas (256 per large message);
//   * counting sort of the slots by bucket (histogram, scan, scatter), one lane per bucket sums its entries, one lane
//     per (L, kind, w) folds sum_d d B_{kind,w,d} with running sums, and one lane group per L combines the windows
//     (R = sum_w [16^w] (W_{0,w} + W_{1,w})) and runs the split Miller loop of (R, H(m)) -> a column of the product
//     tree (the value 1 for an empty R).
#pragma once
#include "rlc.h"
// included by rlcb.h after BLS_ATOMIC_ADD_U32

namespace bls {

constexpr int G1M_BITS = 4;
constexpr int G1M_WIN = 8;                              // 32-bit scalars in 4-bit windows
constexpr uint32_t G1M_ND = (1u << G1M_BITS) - 1;       // non-zero digits per window
constexpr uint32_t G1M_KSTR = 128;                      // bucket indices per (L, kind): 8 x 15 used
constexpr uint32_t G1M_NBL = 2 * G1M_KSTR;              // bucket indices per large message
constexpr uint32_t G1M_NONE = 0xffffffffu;
constexpr uint32_t G1M_MIN = 64;                        // items per message for the G1 MSM (hipbls_rlc_g1_msm_min)

// ---- plan: which messages are large, where their slots start --------------------------------------------------
// cnt[m] items per message -> lid[m] (dense large index or G1M_NONE), lmsg[L] = m, soff[L] = first slot of L
// (soff[nl] = total slots), meta[0] = nl, meta[1] = total slots.  The serial form (host build; the device runs the
// same decisions as a one-workgroup scan, kernels.h k_g1m_plan).
BLS_HD BLS_INLINE void g1m_plan_serial(const uint32_t* cnt, uint64_t n_msgs, uint32_t min, uint32_t* lid,
                                       uint32_t* lmsg, uint32_t* soff, uint32_t* meta) {
  uint32_t nl = 0, tot = 0;
  for (uint64_t m = 0; m < n_msgs; ++m) {
    if (cnt[m] >= min) {
      lid[m] = nl;
      lmsg[nl] = (uint32_t)m;
      soff[nl] = tot;
      ++nl;
      tot += cnt[m];
    } else {
      lid[m] = G1M_NONE;
    }
  }
  soff[nl] = tot;
  meta[0] = nl;
  meta[1] = tot;
}

// item i -> its slot (pos[i]) and the slot's message (slot_l), cursor zeroed per large message
BLS_HD BLS_INLINE void g1m_rank_lane(uint64_t i, const uint32_t* msg_idx, uint64_t n_msgs, const uint32_t* lid,
                                     const uint32_t* soff, uint32_t* cursor, uint32_t* pos, uint32_t* slot_l) {
  const uint32_t m = msg_idx[i];
  const uint32_t L = m < n_msgs ? lid[m] : G1M_NONE;
  if (L == G1M_NONE) {
    pos[i] = G1M_NONE;
    return;
  }
  const uint32_t s = soff[L] + BLS_ATOMIC_ADD_U32(&cursor[L], 1u);
  pos[i] = s;
  slot_l[s] = L;
}

// stage 1's G1 part for an item of a large message (rlcb_items_lane): pk and [x] pk into the slot, with the
// item's scalars; zero scalars when the item already has its final status.  n = the slot capacity (gxp offset).
BLS_HD BLS_INLINE void g1m_store_slot(uint32_t* gpts, uint32_t* gsc, uint64_t n, uint32_t s, bool pending,
                                      const g1a& pk, const g1j& xpk, uint32_t a, uint32_t b) {
  aos_store<24>(gpts, s, &pk.x.v[0]);
  aos_store<36>(gpts + 24 * n, s, &xpk.x.v[0]);
  gsc[2 * (uint64_t)s] = pending ? a : 0u;
  gsc[2 * (uint64_t)s + 1] = pending ? b : 0u;
}

BLS_HD BLS_INLINE uint32_t g1m_digit(uint32_t k, int w) { return (k >> (G1M_BITS * w)) & G1M_ND; }
BLS_HD BLS_INLINE uint64_t g1m_bucket(uint32_t L, int kind, int w, uint32_t d) {
  return (uint64_t)L * G1M_NBL + (uint64_t)kind * G1M_KSTR + (uint64_t)w * G1M_ND + d - 1;
}

// histogram / scatter of slot s's entries (kind 0 with a, kind 1 with b; one per non-zero digit) over its
// message's buckets
BLS_HD BLS_INLINE void g1m_hist_lane(uint64_t s, const uint32_t* meta, const uint32_t* gsc, const uint32_t* slot_l,
                                     uint32_t* bcnt) {
  if (s >= meta[1]) return;
  const uint32_t L = slot_l[s];
  for (int kind = 0; kind < 2; ++kind) {
    const uint32_t k = gsc[2 * s + kind];
    for (int w = 0; w < G1M_WIN; ++w) {
      const uint32_t d = g1m_digit(k, w);
      if (d) BLS_ATOMIC_ADD_U32(&bcnt[g1m_bucket(L, kind, w, d)], 1u);
    }
  }
}
BLS_HD BLS_INLINE void g1m_scatter_lane(uint64_t s, const uint32_t* meta, const uint32_t* gsc,
                                        const uint32_t* slot_l, uint32_t* bcur, uint32_t* list) {
  if (s >= meta[1]) return;
  const uint32_t L = slot_l[s];
  for (int kind = 0; kind < 2; ++kind) {
    const uint32_t k = gsc[2 * s + kind];
    for (int w = 0; w < G1M_WIN; ++w) {
      const uint32_t d = g1m_digit(k, w);
      if (d) list[BLS_ATOMIC_ADD_U32(&bcur[g1m_bucket(L, kind, w, d)], 1u)] = (uint32_t)s;
    }
  }
}

// Bucket sums, load-balanced as the G2 MSM's (rlcb.h msm_run_lane): run lane r adds the G1M_RUN consecutive entries
// [r RUN, (r + 1) RUN) of the bucket-sorted list, bucket run by bucket run (kind 1 = [x] pk, Jacobian, full additions;
// kind 0 = pk, affine, mixed additions); a bucket wholly inside the range goes to B, a bucket cut by the range's
// start or end leaves a partial in P (slot 0 = the lane's first run, 1 = its last) for g1m_fix_lane.  B, P: Jacobian,
// 36 words, AoS.  boff: exclusive offsets over all nl_max * G1M_NBL indices (entries = boff[meta[0] * G1M_NBL]).
// Launched for g1m_run_lanes(n) lanes, the bound for 16 entries per slot.
constexpr int G1M_RUN = 64;
BLS_HD BLS_INLINE uint64_t g1m_run_lanes(uint64_t n) { return (2 * (uint64_t)G1M_WIN * n + G1M_RUN - 1) / G1M_RUN; }

BLS_HD BLS_INLINE void g1m_run_lane(uint64_t r, const uint32_t* meta, const uint32_t* boff, const uint32_t* list,
                                    const uint32_t* gpts, uint64_t n, uint32_t* B, uint32_t* P) {
  const uint64_t nbk = (uint64_t)meta[0] * G1M_NBL;
  if (nbk == 0) return;
  const uint64_t total = boff[nbk], k0 = r * G1M_RUN;
  if (k0 >= total) return;
  const uint64_t k1 = k0 + G1M_RUN < total ? k0 + G1M_RUN : total;
  uint64_t lo = 0, hi = nbk;  // the bucket of entry k0: boff[lo] <= k0 < boff[hi]
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (boff[mid] <= k0)
      lo = mid;
    else
      hi = mid;
  }
  // One addition per iteration on every lane (a loop per bucket run made the wave wait for each lane's longest run
  // in turn): the point of entry k + 1 is prefetched in its bucket's kind before entry k's addition; the kind is the
  // same across a wave except where its 2,048 entries straddle a kind boundary.
  uint64_t b = lo, end = boff[b + 1];
  bool kind = ((b / G1M_KSTR) & 1) != 0;
  int slot = 0;
  const uint32_t* gxp = gpts + 24 * n;
  g1j q;
  if (kind)
    aos_load<36>(&q.x.v[0], gxp, list[k0]);
  else
    aos_load<24>(&q.x.v[0], gpts, list[k0]);
  g1j acc;
  jac_set_inf(acc);
  for (uint64_t k = k0; k < k1; ++k) {
    const g1j cur = q;
    const bool kc = kind;
    uint64_t nb = b;
    if (k + 1 < k1) {
      if (k + 1 == end) {
        ++nb;
        while (boff[nb + 1] <= k + 1) ++nb;  // the next non-empty bucket
      }
      const bool kn = ((nb / G1M_KSTR) & 1) != 0;
      if (kn)
        aos_load<36>(&q.x.v[0], gxp, list[k + 1]);
      else
        aos_load<24>(&q.x.v[0], gpts, list[k + 1]);
    }
    g1j x = acc, y;
    if (kc) {
      jac_add_body(y, x, cur);
    } else {
      g1a ca;
      ca.x = cur.x;
      ca.y = cur.y;
      jac_add_aff_body(y, x, ca);
    }
    acc = y;
    if (k + 1 == end || k + 1 == k1) {  // bucket b's run in this range ends here
      if (boff[b] >= k0 && end <= k1)
        aos_store<36>(B, b, &acc.x.v[0]);
      else
        aos_store<36>(P, 2 * r + slot, &acc.x.v[0]);
      slot = 1;
      jac_set_inf(acc);
      b = nb;
      end = boff[b + 1];
      kind = ((b / G1M_KSTR) & 1) != 0;
    }
  }
}

// bucket b after the run lanes (as rlcb.h msm_fix_lane): infinity when empty, written already when one run lane holds
// all its entries, otherwise the sum of its partials.
BLS_HD BLS_INLINE void g1m_fix_lane(uint64_t b, const uint32_t* meta, const uint32_t* boff, uint32_t* B,
                                    const uint32_t* P) {
  if (b >= (uint64_t)meta[0] * G1M_NBL) return;
  const uint64_t k0 = boff[b], k1 = boff[b + 1];
  g1j acc;
  if (k0 == k1) {
    jac_set_inf(acc);
    aos_store<36>(B, b, &acc.x.v[0]);
    return;
  }
  const uint64_t a = k0 / G1M_RUN, e = (k1 - 1) / G1M_RUN;
  if (a == e) return;
  aos_load<36>(&acc.x.v[0], P, 2 * a + (k0 == a * G1M_RUN ? 0 : 1));
  for (uint64_t l = a + 1; l <= e; ++l) {
    g1j p, x = acc, y;
    aos_load<36>(&p.x.v[0], P, 2 * l);
    jac_add_body(y, x, p);
    acc = y;
  }
  aos_store<36>(B, b, &acc.x.v[0]);
}

// q = (L, kind, w): W_q = sum_{d=1..15} d B_{L,kind,w,d} by running sums (top digit first): R = sum_{d' >= d} B_d',
// T = sum_d R -- 30 additions of latency per lane (a lane per kind, not one for both: the fold is latency-bound)
constexpr uint32_t G1M_NFOLD = 2 * G1M_WIN;  // fold lanes (window sums) per large message
BLS_HD BLS_INLINE void g1m_fold_lane(uint64_t q, const uint32_t* meta, const uint32_t* B, uint32_t* Wv) {
  if (q >= (uint64_t)meta[0] * G1M_NFOLD) return;
  const uint32_t L = (uint32_t)(q / G1M_NFOLD);
  const int kind = (int)((q / G1M_WIN) & 1), w = (int)(q % G1M_WIN);
  g1j R, T;
  jac_set_inf(R);
  jac_set_inf(T);
  for (uint32_t d = G1M_ND; d >= 1; --d) {
    g1j b;
    aos_load<36>(&b.x.v[0], B, g1m_bucket(L, kind, w, d));
    g1j x = R, y;
    jac_add_body(y, x, b);
    R = y;
    g1j u = T, v;
    jac_add_body(v, u, R);
    T = v;
  }
  aos_store<36>(Wv, q, &T.x.v[0]);
}

// window w of message L: W_{L,0,w} + W_{L,1,w}
BLS_HD BLS_INLINE void g1m_window(g1j& W, const uint32_t* Wv, uint64_t L, int w) {
  g1j a, b;
  aos_load<36>(&a.x.v[0], Wv, L * G1M_NFOLD + (uint64_t)w);
  aos_load<36>(&b.x.v[0], Wv, L * G1M_NFOLD + G1M_WIN + (uint64_t)w);
  jac_add(W, a, b);
}

// R_L = sum_w [16^w] W_{L,w} (Horner from the top window)
BLS_HD BLS_INLINE void g1m_combine(g1j& R, const uint32_t* Wv, uint64_t L) {
  g1m_window(R, Wv, L, G1M_WIN - 1);
  for (int w = G1M_WIN - 2; w >= 0; --w) {
    for (int k = 0; k < G1M_BITS; ++k) {
      g1j t;
      jac_dbl_body(t, R);
      R = t;
    }
    g1j t;
    g1m_window(t, Wv, L, w);
    g1j x = R, y;
    jac_add(y, x, t);
    R = y;
  }
}

// the windows' fallback after a failed batch check needs [r_i] pk_i per item: from the slot (Shamir, as stage 1)
BLS_HD BLS_INLINE void g1m_item_rpk(g1j& rp, const uint32_t* gpts, uint64_t n, const uint32_t* gsc, uint32_t s) {
  g1a pk;
  g1j pj, xj;
  aos_load<24>(&pk.x.v[0], gpts, s);
  aos_load<36>(&xj.x.v[0], gpts + 24 * n, s);
  jac_from_aff(pj, pk);
  jac_mul2_u32(rp, pj, xj, gsc[2 * (uint64_t)s], gsc[2 * (uint64_t)s + 1]);
}

// the Miller value of (R_L, H(m_L)) on one lane into column col of F (host build; the device splits it over a lane
// pair, verify_lat.hip k_g1m_miller8); the value 1 for L >= nl or an empty R
template <int S>
BLS_HD BLS_INLINE void g1m_miller_lane(const f12l<S>& Lf, uint64_t L, const uint32_t* meta, const uint32_t* lmsg,
                                       const uint32_t* Wv, const uint32_t* H, uint64_t hstride, const uint32_t* hslot,
                                       uint32_t* F, uint64_t col, uint64_t fstride) {
  fp12 f;
  fp12_set_one(f);
  if (L < meta[0]) {
    g1j R;
    g1m_combine(R, Wv, L);
    if (!jac_is_inf(R)) {
      g1a P[1];
      g2a Q[1];
      jac_to_aff(P[0], R);
      soa_load<48>(&Q[0].x.c0.v[0], H, hstride, h_col(hslot, lmsg[L]));
      miller_loop_multi_l<1>(f, Lf, P, Q, 1);
    }
  }
  soa_store<144>(F, fstride, col, &f.c0.c0.c0.v[0]);
}

}  // namespace bls
