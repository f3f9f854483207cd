// Latency-bound kernels on twice the lanes, with every Fp2 product and square split across twin lanes:
//   * the drop-in latency path: tbls.Verify for batches far below one wave of work per SIMD (the unpatched callers'
//     n = 1 calls, /root/reference/core/parsigex/parsigex.go:86-91 and core/validatorapi/validatorapi.go:246-283), on
//     EIGHT lanes per item (VERDICT r03 "Next round" 8): the lane-quad Verify of kernels.h (k_verify_prep +
//     k_verify_pair_lq4, lg2.h lq4_verify) with every Fp2 product and square split across lanes l and l ^ 4
//     (field.h fp2p_*, tower.h), so the quad's lanes 0-3 and their twins 4-7 hold the same values and each does half
//     of every Fp2 product;
//   * the batch-wide RLC check's serial tail (rlcb.h): the (-g1, S) Miller value, the verdict's final
//     exponentiation, and the Miller value of each large message's G1 MSM sum (g1msm.h).
// Same formulas, same results; ~0.7x the latency of the Fp2-bound chains (hash to G2, Miller loops, final
// exponentiation: profiles/r04/latency_sweep_quads_octets.json).
//
// Everything here lives in namespace bls_fp2p (the kernel headers are included with `bls` renamed), so its inline
// functions never meet the main translation unit's on the host side; hipbls.hip declares and launches the two kernels.
#define BLS_FP2_PAIR 1
#define bls bls_fp2p
#include <hip/hip_runtime.h>

#include "race.h"

#include "lg2.h"
#include "rlcb.h"

namespace bls {

constexpr int kOctBlock = 64;

// ---------------------------------------------------------------- the hash's cofactor clearing on a lane quad
// G2 doubling (curve.h jac_dbl_body, dbl-2009-l) with its seven Fp2 products dealt out over the quad's lanes
// (q = lane & 3): level 1 X^2 | Y^2 | Y Z, level 2 B^2 | (X + B)^2 | E^2, level 3 E (D - X3) on every lane; each level's
// products are broadcast to the quad (lg2.h quad_bcast).  Three products of latency instead of seven; every lane
// ends with the same point.  All four lanes (and, here, their Fp2 twins) must be active.
__device__ __forceinline__ void g2_dbl_quad(g2j& r, const g2j& p, int q) {
  const uint32_t q1 = q == 1 ? ~0u : 0u, q2 = q == 2 ? ~0u : 0u;
  fp2 x, y, o;
  x = sel(q2, p.y, sel(q1, p.y, p.x));
  y = sel(q2, p.z, sel(q1, p.y, p.x));
  fp2_mul(o, x, y);  // X^2 | Y^2 | Y Z
  const fp2 A = quad_bcast<0>(o), B = quad_bcast<1>(o), YZ = quad_bcast<2>(o);
  fp2 XB, E;
  fp2_add(XB, p.x, B);
  fp2_add(E, A, A);
  fp2_add(E, E, A);
  x = sel(q2, E, sel(q1, XB, B));
  fp2_mul(o, x, x);  // C = B^2 | (X + B)^2 | F = E^2
  const fp2 C = quad_bcast<0>(o), T = quad_bcast<1>(o), Fv = quad_bcast<2>(o);
  fp2 t, D, x3, c8;
  fp2_sub(t, T, A);
  fp2_sub(t, t, C);
  fp2_add(D, t, t);
  fp2_sub(x3, Fv, D);
  fp2_sub(x3, x3, D);
  fp2_sub(t, D, x3);
  fp2_mul(t, E, t);
  fp2_add(c8, C, C);
  fp2_add(c8, c8, c8);
  fp2_add(c8, c8, c8);
  fp2_sub(r.y, t, c8);
  fp2_add(r.z, YZ, YZ);
  r.x = x3;
}

// G2 addition (curve.h jac_add_body, add-2007-bl: 11 products + 5 squarings) dealt out over the quad in five levels
// of one product per lane, each level broadcast to the quad:
//   1: Z1^2 | Z2^2 | Y1 Z2 | Y2 Z1          2: U1 = X1 Z2^2 | U2 = X2 Z1^2 | S1 = Y1 Z2^3 | S2 = Y2 Z1^3
//   3: I = (2H)^2 | R^2 | (Z1 + Z2)^2        4: J = H I | V = U1 I | Z3 = ((Z1 + Z2)^2 - Z1^2 - Z2^2) H
//   5: R (V - X3) | S1 J
// Five products of latency instead of sixteen; squarings as products of equal operands (the same canonical values).
// The exceptional cases (an input at infinity, H = 0) take jac_add on every lane: the values are the same on all
// four lanes, so those branches are quad-uniform.  All four lanes (and their Fp2 twins) must be active.
__device__ __forceinline__ void g2_add_quad(g2j& r, const g2j& p, const g2j& qp, int q) {
  if (jac_is_inf(p) || jac_is_inf(qp)) {
    jac_add(r, p, qp);
    return;
  }
  const uint32_t q1 = q == 1 ? ~0u : 0u, q2 = q == 2 ? ~0u : 0u, q3 = q == 3 ? ~0u : 0u;
  fp2 x, y, o;
  x = sel(q3, qp.y, sel(q2, p.y, sel(q1, qp.z, p.z)));
  y = sel(q3, p.z, sel(q2, qp.z, sel(q1, qp.z, p.z)));
  fp2_mul(o, x, y);
  const fp2 z1z1 = quad_bcast<0>(o), z2z2 = quad_bcast<1>(o), s1a = quad_bcast<2>(o), s2a = quad_bcast<3>(o);
  x = sel(q3, s2a, sel(q2, s1a, sel(q1, qp.x, p.x)));
  y = sel(q3, z1z1, sel(q2, z2z2, sel(q1, z1z1, z2z2)));
  fp2_mul(o, x, y);
  const fp2 u1 = quad_bcast<0>(o), u2 = quad_bcast<1>(o), s1 = quad_bcast<2>(o), s2 = quad_bcast<3>(o);
  fp2 h, rr;
  fp2_sub(h, u2, u1);
  fp2_sub(rr, s2, s1);
  if (fp2_is_zero(h)) {  // the same on all four lanes
    if (fp2_is_zero(rr))
      jac_dbl(r, p);
    else
      jac_set_inf(r);
    return;
  }
  fp2_add(rr, rr, rr);
  fp2 h2, zs;
  fp2_add(h2, h, h);
  fp2_add(zs, p.z, qp.z);
  x = sel(q2, zs, sel(q1, rr, h2));
  fp2_mul(o, x, x);
  const fp2 i = quad_bcast<0>(o), r2 = quad_bcast<1>(o), zz = quad_bcast<2>(o);
  fp2 zc;
  fp2_sub(zc, zz, z1z1);
  fp2_sub(zc, zc, z2z2);
  x = sel(q2, zc, sel(q1, u1, h));
  y = sel(q2, h, i);
  fp2_mul(o, x, y);
  const fp2 j = quad_bcast<0>(o), v = quad_bcast<1>(o), z3 = quad_bcast<2>(o);
  fp2 x3, t;
  fp2_sub(x3, r2, j);
  fp2_sub(x3, x3, v);
  fp2_sub(x3, x3, v);
  fp2_sub(t, v, x3);
  x = sel(q1, s1, rr);
  y = sel(q1, j, t);
  fp2_mul(o, x, y);
  const fp2 y3a = quad_bcast<0>(o), s1j = quad_bcast<1>(o);
  fp2 y3, s1j2;
  fp2_add(s1j2, s1j, s1j);
  fp2_sub(y3, y3a, s1j2);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// [|x|] p with the doublings and the additions (at |x|'s five set bits below the top) on the quad
__device__ void g2_mul_xabs_quad(g2j& r, const g2j& p_in, int q) {
  const g2j p = p_in;
  g2j acc = p;
  for (int i = 62; i >= 0; --i) {
    if ((i & 3) == 3) BLS_RACE_POLL();
    g2j t;
    g2_dbl_quad(t, acc, q);
    acc = t;
    if ((X_ABS >> i) & 1ull) {
      g2j u = acc;
      g2_add_quad(acc, u, p, q);
    }
  }
  r = acc;
}

// curve.h g2_clear_cofactor (Budroni-Pintore) with its two [x] multiplications, its doubling and its additions on the
// quad
__device__ void g2_clear_cofactor_quad(g2j& r, const g2j& p_in, int q) {
  const g2j p = p_in;
  g2j t1, t2, t3, np, nt1, nt2, u;
  g2_mul_xabs_quad(t1, p, q);
  jac_neg(t1, t1);  // [x] P
  g2_psi(t2, p);
  g2_dbl_quad(t3, p, q);
  g2_psi2(t3, t3);
  jac_neg(nt2, t2);
  u = t3;
  g2_add_quad(t3, u, nt2, q);  // psi^2(2P) - psi(P)
  u = t2;
  g2_add_quad(t2, t1, u, q);   // [x] P + psi(P)
  g2_mul_xabs_quad(t2, t2, q);
  jac_neg(t2, t2);
  u = t3;
  g2_add_quad(t3, u, t2, q);
  jac_neg(nt1, t1);
  u = t3;
  g2_add_quad(t3, u, nt1, q);
  jac_neg(np, p);
  g2_add_quad(r, t3, np, q);
}

// Stage 1, eight lanes per item (t >> 3), three roles per set of workgroups (uniform per workgroup, so they run side
// by side on different SIMDs): decode + check the key, decode the signature, hash the message (lanes 0/1 of each
// quad split the two SSWU maps, lg2.h hash_to_g2_pair_sum, and the quad clears the cofactor).  The decode codes go
// to ws + 120 n (two words per item); k_verify_pair_lq8 composes the status in herumi's order.  ws: pk (24 x n),
// H(m) (48 x n), sig (48 x n), SoA.
// Replicas: `replicas` consecutive workgroups run the same original workgroup (race word race[role], epoch).
__global__ void __launch_bounds__(kOctBlock) k_verify_prep8(const uint8_t* __restrict__ pks,
                                                            const uint8_t* __restrict__ msgs,
                                                            const uint64_t* __restrict__ offs,
                                                            const uint8_t* __restrict__ sigs, uint64_t n,
                                                            uint32_t* __restrict__ ws, int32_t* __restrict__ status,
                                                            uint32_t replicas, uint32_t* __restrict__ race,
                                                            uint32_t epoch) {
  (void)status;  // k_verify_pair_lq8 writes every status
  const uint64_t nb = (8 * n + kOctBlock - 1) / kOctBlock;
  const uint64_t rb = blockIdx.x / replicas;  // the original workgroup this copy runs
  const uint64_t role = rb / nb;              // 0 key, 1 signature, 2 hash: uniform per workgroup
  bls_race::init(replicas > 1 ? race + role : nullptr, epoch);
  const uint64_t t = (rb - role * nb) * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 3;
  if (i >= n) return;  // the same on all eight lanes
  const bool lead = (t & 7) == 0;
  int32_t* codes = (int32_t*)(ws + 120 * n);
  if (role == 2) {
    const uint32_t m = (t & 1) ? ~0u : 0u;
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j sum, hj;
    hash_to_g2_pair_sum(sum, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43, m);
    g2_clear_cofactor_quad(hj, sum, (int)(t & 3));
    BLS_RACE_POLL();
    g2a hm;
    jac_to_aff(hm, hj);
    if (lead) soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
    bls_race::finish();
    return;
  }
  if (role == 0) {
    g1a pk;
    const int dp = g1_decompress(pk, pks + 48 * i, true);
    if (lead) {
      codes[2 * i] = dp;
      if (dp == DEC_OK) soa_store<24>(ws, n, i, &pk.x.v[0]);
    }
    bls_race::finish();
    return;
  }
  g2a sig;
  const int ds = g2_decompress(sig, sigs + 96 * i, false);  // G2 membership: from the signature's Miller loop
  if (lead) {
    codes[2 * i + 1] = ds;
    if (ds == DEC_OK) soa_store<48>(ws + 72 * n, n, i, &sig.x.c0.v[0]);
  }
  bls_race::finish();
}

// FastAggregateVerify's stage 1 for a few groups (tbls/herumi.go:315-339; hipbls.hip launch_fav, the sync committee's
// one aggregate per slot), eight lanes per unit: every key of every group decoded + subgroup-tested (pts: affine SoA
// with stride nkeys, kcode: DEC_* per key), beside each group's signature decode and message hash exactly as
// k_verify_prep8's roles 1 and 2 (ws: H(m) at 24 G, sig at 72 G, the signature's code at word 2 g + 1 of 120 G).
// Workgroups: the key blocks, then the signature blocks, then the hash blocks.  Not raced.
__global__ void __launch_bounds__(kOctBlock) k_fav_prep8(const uint8_t* __restrict__ pks, uint64_t nkeys,
                                                         const uint8_t* __restrict__ sigs,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ moffs, uint64_t G,
                                                         uint32_t* __restrict__ pts, int32_t* __restrict__ kcode,
                                                         uint32_t* __restrict__ ws) {
  bls_race::init(nullptr, 0u);
  const uint64_t nbk = (8 * nkeys + kOctBlock - 1) / kOctBlock;
  const uint64_t nbg = (8 * G + kOctBlock - 1) / kOctBlock;
  uint64_t b = blockIdx.x;
  int role = 0;  // 0 key, 1 signature, 2 hash: uniform per workgroup
  if (b >= nbk) {
    b -= nbk;
    role = b < nbg ? 1 : 2;
    if (role == 2) b -= nbg;
  }
  const uint64_t t = b * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 3;
  const bool lead = (t & 7) == 0;
  if (role == 0) {
    if (i >= nkeys) return;  // the same on all eight lanes
    g1a pk;
    const int dp = g1_decompress(pk, pks + 48 * i, true);
    if (lead) {
      kcode[i] = dp;
      if (dp == DEC_OK) soa_store<24>(pts, nkeys, i, &pk.x.v[0]);
    }
    return;
  }
  if (i >= G) return;
  if (role == 2) {
    const uint32_t m = (t & 1) ? ~0u : 0u;
    const uint64_t o0 = moffs[i], o1 = moffs[i + 1];
    g2j sum, hj;
    hash_to_g2_pair_sum(sum, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43, m);
    g2_clear_cofactor_quad(hj, sum, (int)(t & 3));
    g2a hm;
    jac_to_aff(hm, hj);
    if (lead) soa_store<48>(ws + 24 * G, G, i, &hm.x.c0.v[0]);
    return;
  }
  g2a sig;
  const int ds = g2_decompress(sig, sigs + 96 * i, false);  // G2 membership: from the check's Miller loop
  if (lead) {
    ((int32_t*)(ws + 120 * G))[2 * i + 1] = ds;
    if (ds == DEC_OK) soa_store<48>(ws + 72 * G, G, i, &sig.x.c0.v[0]);
  }
}

#ifndef BLS_LQ8_XCD_PROBE
#define BLS_LQ8_XCD_PROBE 0
#endif
#if BLS_LQ8_XCD_PROBE
// Experiment build only (scripts/xcd_lq8_probe.py): every workgroup runs 8 times, once per XCD, each copy recording its
// XCC id and its start / end on the 100 MHz real-time counter, to see whether the check's duration depends on the XCD
// its workgroup lands on.
__device__ uint64_t g_xcd_probe[64 * 4];
#endif

// Stage 2, eight lanes per item: the status from the decode codes in herumi's order (key, then signature, then the
// infinity cases), then lq4_verify on lanes 0-3 (q = t & 3) and, as their Fp2 twins, on 4-7.
__global__ void __launch_bounds__(kOctBlock) k_verify_pair_lq8(const uint32_t* __restrict__ ws, uint64_t n,
                                                               int32_t* __restrict__ status, uint32_t replicas,
                                                               uint32_t* __restrict__ race, uint32_t epoch) {
  bls_race::init(replicas > 1 ? race + 3 : nullptr, epoch);
#if BLS_LQ8_XCD_PROBE
  const uint64_t t0_probe = __builtin_amdgcn_s_memrealtime();
  const uint64_t t = (blockIdx.x >> 3) * (uint64_t)blockDim.x + threadIdx.x;
  struct ProbeEnd {
    uint64_t t0;
    __device__ ~ProbeEnd() {
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      uint32_t x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      if (threadIdx.x == 0 && blockIdx.x < 64) {
        g_xcd_probe[4 * blockIdx.x] = x;
        g_xcd_probe[4 * blockIdx.x + 1] = t0;
        g_xcd_probe[4 * blockIdx.x + 2] = t1;
      }
    }
  } probe_end{t0_probe};
#else
  const uint64_t t = (blockIdx.x / replicas) * (uint64_t)blockDim.x + threadIdx.x;
#endif
  const uint64_t i = t >> 3;
  if (i >= n) return;  // the same on all eight lanes
  const int32_t* codes = (const int32_t*)(ws + 120 * n);
  const int dp = codes[2 * i], ds = codes[2 * i + 1];
  const bool lead = (t & 7) == 0;
  g2a sig;
  if (ds == DEC_OK) soa_load<48>(&sig.x.c0.v[0], ws + 72 * n, n, i);
  int st = RLC_PENDING;
  if (dp == DEC_BAD)
    st = HIPBLS_ERR_PUBKEY;
  else if (ds == DEC_BAD)
    st = HIPBLS_ERR_SIGNATURE;
  else if (dp == DEC_INF || ds == DEC_INF)
    st = verify_inf_status(ds, sig);  // KeyValidate / e(pk, H) != 1
  if (st != RLC_PENDING) {
    if (lead) status[i] = st;
    return;
  }
  g1a pk;
  g2a hm;
  soa_load<24>(&pk.x.v[0], ws, n, i);
  soa_load<48>(&hm.x.c0.v[0], ws + 24 * n, n, i);
  st = lq4_verify(pk, hm, sig, (int)(t & 3));
  if (lead) status[i] = st;
  bls_race::finish();
}

// ---------------------------------------------------------------- the batch-wide RLC check's tail (rlcb.h)
// The Miller value of (-g1, S), S = W0 + [2^16] W1 from the MSM's window sums (rlcb.h msm_combine): lanes 0/1 split
// the loop (lg2.h miller_loop_split), lanes 4/5 are their Fp2 twins (2, 3, 6, 7 repeat them); 144 words to Fs.
__global__ void __launch_bounds__(kOctBlock) k_rlcb_sfactor8(const uint32_t* __restrict__ W, uint32_t* __restrict__ Fs) {
  bls_race::init(nullptr, 0);  // not raced (LDS is not zero-initialized)
  const int t = threadIdx.x;
  if (t >= 8) return;
  const uint32_t m = (t & 1) ? ~0u : 0u;
  g2j W0, W1, S;
  for (int k = 0; k < 72; ++k) {
    (&W0.x.c0.v[0])[k] = W[k];
    (&W1.x.c0.v[0])[k] = W[72 + k];
  }
  msm_combine(S, W0, W1);
  fp12 f;
  if (jac_is_inf(S)) {  // the same on all eight lanes
    fp12_set_one(f);
  } else {
    g1a P;
    P.x = G1_GEN_X;
    P.y = G1_NEG_GEN_Y;
    g2a Q;
    jac_to_aff(Q, S);
    fp6 h;
    miller_loop_split(h, P, Q, m);
    fp12h_gather(f, h, m);
  }
  if (t == 0)
    for (int k = 0; k < 144; ++k) Fs[k] = (&f.c0.c0.c0.v[0])[k];
}

// The verdict: the product tree's value (Ftot) times the (-g1, S) value (Fs) and the final exponentiation on a lane
// quad (lanes 0-3, lg2.h fp12q_mul / final_exponentiation_quad) with Fp2 twins on 4-7; flag[0] = 1 when it is 1.
__global__ void __launch_bounds__(kOctBlock) k_rlcb_final8(const uint32_t* __restrict__ Ftot,
                                                           const uint32_t* __restrict__ Fs, int32_t* __restrict__ flag) {
  bls_race::init(nullptr, 0);  // not raced (LDS is not zero-initialized)
  const int t = threadIdx.x;
  if (t >= 8) return;
  fp12 a, b, r, e;
  for (int k = 0; k < 144; ++k) {
    (&a.c0.c0.c0.v[0])[k] = Fs[k];
    (&b.c0.c0.c0.v[0])[k] = Ftot[k];
  }
  const quad_m qm(t & 3);
  fp12q_mul(r, a, b, qm);
  final_exponentiation_quad(e, r, qm);
  const bool ok = fp12_is_one(e);
  if (t == 0) flag[0] = ok ? 1 : 0;
}

// Eight lanes per large message L < nl_max (g1msm.h): R_L from the window sums, the Miller value of (R_L, H(m_L))
// split over lanes 0/1 with Fp2 twins 4/5 (2, 3, 6, 7 repeat them); lane 0 writes column col0 + L of F.  The value 1
// for L >= nl or an empty R.
__global__ void __launch_bounds__(kOctBlock) k_g1m_miller8(uint64_t nl_max, const uint32_t* __restrict__ meta,
                                                           const uint32_t* __restrict__ lmsg,
                                                           const uint32_t* __restrict__ Wv,
                                                           const uint32_t* __restrict__ H, uint64_t hstride,
                                                           const uint32_t* __restrict__ hslot, uint32_t* __restrict__ F,
                                                           uint64_t col0, uint64_t fstride) {
  bls_race::init(nullptr, 0);  // not raced (LDS is not zero-initialized)
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t L = t >> 3;
  if (L >= nl_max) return;  // the same on all eight lanes
  const uint32_t m = (t & 1) ? ~0u : 0u;
  fp12 f;
  fp12_set_one(f);
  if (L < meta[0]) {
    g1j R;
    g1m_combine(R, Wv, L);
    if (!jac_is_inf(R)) {
      g1a P;
      g2a Q;
      jac_to_aff(P, R);
      soa_load<48>(&Q.x.c0.v[0], H, hstride, h_col(hslot, lmsg[L]));
      fp6 h;
      miller_loop_split(h, P, Q, m);
      fp12h_gather(f, h, m);
    }
  }
  if ((t & 7) == 0) soa_store<144>(F, fstride, col0 + L, &f.c0.c0.c0.v[0]);
}

}  // namespace bls

#if BLS_LQ8_XCD_PROBE
extern "C" int hipbls_debug_xcd_probe(uint64_t* out256) {
  return hipMemcpyFromSymbol(out256, HIP_SYMBOL(bls_fp2p::g_xcd_probe), sizeof(uint64_t) * 256) == hipSuccess ? 0 : 17;
}
#endif
