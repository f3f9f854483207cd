// Two-lane groups for the pairing check (BASELINE.json north star: "one lane-group per pairing with
// wavefront-level reductions").  Lanes 2i and 2i+1 of a wave cooperate on one pairing-product check:
//
//   * Miller loop: each lane runs the Miller loop of its own pairs (lane 0: e(pk, H(m)), lane 1: e(-g1, sig) for a
//     Verify; pairs of equal parity for a multi-pairing), so the two loops run side by side instead of one after
//     the other.  Same instruction stream on both lanes, different data (SIMT-uniform).
//   * The two Miller values are combined into ONE Fp12 held split across the pair: the even lane owns c0, the odd
//     lane owns c1 (Fp12 = Fp6[w]).  Halves are exchanged with DPP quad_perm [1,0,3,2] moves (one VALU instruction
//     per dword, no LDS), which need both lanes of a pair active: every exchange sits in pair-uniform control flow.
//   * The final exponentiation runs on the split value: each lane computes its own half of every product
//     (Fp12 products: two Fp6 products per lane, schoolbook; the exponentiations by |x| as Karabina's compressed
//     squarings with three Fp2 squarings per lane instead of six), so its latency is roughly halved.  The
//     inversion of the easy part is computed redundantly on both lanes from the gathered value.
//   * Lane quads (miller_loop_split, lq4_verify): for batches that leave lanes idle, ONE Miller loop is split across
//     a pair (the Fp12 squaring and line products halved, the doubling step's products dealt out), a quad runs a
//     Verify's two loops on its two pairs, and the final exponentiation is dealt out over the quad: n = 1 Verify
//     23.8 -> 18.6 ms, C3 359k -> 439k aggregates/s (profiles/r03_pair_sweep_dblsplit.txt).
//
// Semantics are those of pairing_check_verify / the RLC checks (ops.h, rlc.h): the same formulas, the same e^3
// final exponentiation, so a split check and a single-lane check accept exactly the same inputs.  Device-only
// (DPP); parity is covered by the GPU tests against the single-lane kernels and the oracle.
#pragma once
#include "rlc.h"

#ifndef BLS_HEX
#define BLS_HEX 0
#endif

namespace bls {

#if defined(__HIPCC__)

// Replica race hook (verify_lat.hip): a latency kernel launched as several replicas of the same work, one per XCD,
// polls here at coarse steps and ends a replica once another has finished (the first finisher wins; every replica
// computes the same result).  An empty statement in every other build.
#ifndef BLS_RACE_POLL
#define BLS_RACE_POLL() ((void)0)
#endif

// Partner lane's value (lane ^ 1).  Both lanes of the pair must be active.
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1 /* quad_perm [1,0,3,2] */, 0xF, 0xF, false);
#else
  return v;  // host pass of a device function: never executed
#endif
}
template <int N>
__device__ __forceinline__ void pair_swap_words(uint32_t* d, const uint32_t* s) {
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = pair_swap(s[i]);
}
__device__ __forceinline__ void pair_swap(fp2& d, const fp2& s) { pair_swap_words<24>(&d.c0.v[0], &s.c0.v[0]); }
__device__ __forceinline__ void pair_swap(fp6& d, const fp6& s) { pair_swap_words<72>(&d.c0.c0.v[0], &s.c0.c0.v[0]); }

// Lane-parity selects: m = ~0 on the odd lane, 0 on the even one.  Bitwise (v_bfi_b32), never a VOP2 cndmask.
template <int N>
__device__ __forceinline__ void sel_words(uint32_t* d, uint32_t m, const uint32_t* if_odd, const uint32_t* if_even) {
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = (m & if_odd[i]) | (~m & if_even[i]);
}
__device__ __forceinline__ fp2 sel(uint32_t m, const fp2& if_odd, const fp2& if_even) {
  fp2 r;
  sel_words<24>(&r.c0.v[0], m, &if_odd.c0.v[0], &if_even.c0.v[0]);
  return r;
}
__device__ __forceinline__ fp6 sel(uint32_t m, const fp6& if_odd, const fp6& if_even) {
  fp6 r;
  sel_words<72>(&r.c0.c0.v[0], m, &if_odd.c0.c0.v[0], &if_even.c0.c0.v[0]);
  return r;
}

// ---------------------------------------------------------------- sixteen lanes per item (verify_hex.hip, BLS_HEX)
// The split-Fp2 build run on sixteen lanes per item: lanes 0-7 and 8-15 of each group hold the same octet state and
// run the same code; the Fp6 products and the compressed squarings' Fp2 squarings are dealt out over the two halves
// (lane ^ 8, one DPP row_ror:8 per dword).  Every other step runs redundantly on both halves.  All sixteen lanes must
// be active.
#if BLS_HEX
__device__ __forceinline__ uint32_t hx_mask() {  // ~0 on lanes 8-15 of each group of sixteen
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  return (lane & 8u) ? ~0u : 0u;
}
__device__ __forceinline__ uint32_t hx_xchg(uint32_t v) {  // lane ^ 8 within the row of sixteen
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128 /* row_ror:8 */, 0xF, 0xF, false);
#else
  return v;
#endif
}
__device__ __forceinline__ fp2 hx_xchg(const fp2& s) {
  fp2 d;
#pragma unroll
  for (int i = 0; i < 24; ++i) (&d.c0.v[0])[i] = hx_xchg((&s.c0.v[0])[i]);
  return d;
}
// tower.h fp6_mul (Karatsuba, six Fp2 products) with the products dealt out: the low half forms a0 b0, a1 b1, a2 b2,
// the high half (a1 + a2)(b1 + b2), (a0 + a1)(b0 + b1), (a0 + a2)(b0 + b2); one exchange, then both halves combine
// them as fp6_mul does.  Three products of latency instead of six; the same canonical result.
__device__ __forceinline__ void fp6_mul_hx(fp6& r, const fp6& a_in, const fp6& b_in) {
  const fp6 a = a_in, b = b_in;
  const uint32_t h = hx_mask();
  fp2 s0, s1, p0, p1, p2;
  fp2_add_lazy(s0, a.c1, a.c2);
  fp2_add_lazy(s1, b.c1, b.c2);
  fp2_mul(p0, sel(h, s0, a.c0), sel(h, s1, b.c0));
  fp2_add_lazy(s0, a.c0, a.c1);
  fp2_add_lazy(s1, b.c0, b.c1);
  fp2_mul(p1, sel(h, s0, a.c1), sel(h, s1, b.c1));
  fp2_add_lazy(s0, a.c0, a.c2);
  fp2_add_lazy(s1, b.c0, b.c2);
  fp2_mul(p2, sel(h, s0, a.c2), sel(h, s1, b.c2));
  const fp2 o0 = hx_xchg(p0), o1 = hx_xchg(p1), o2 = hx_xchg(p2);
  const fp2 t0 = sel(h, o0, p0), t1 = sel(h, o1, p1), t2 = sel(h, o2, p2);
  const fp2 m12 = sel(h, p0, o0), m01 = sel(h, p1, o1), m02 = sel(h, p2, o2);
  fp2 u0, u1, u2, x2;
  fp2_sub(u0, m12, t1);
  fp2_sub(u0, u0, t2);
  fp2_mul_xi(u0, u0);
  fp2_add(u0, u0, t0);
  fp2_sub(u1, m01, t0);
  fp2_sub(u1, u1, t1);
  fp2_mul_xi(x2, t2);
  fp2_add(u1, u1, x2);
  fp2_sub(u2, m02, t0);
  fp2_sub(u2, u2, t2);
  fp2_add(u2, u2, t1);
  r.c0 = u0;
  r.c1 = u1;
  r.c2 = u2;
}
#define LG2_FP6_MUL fp6_mul_hx
#else
#define LG2_FP6_MUL fp6_mul
#endif

// ---------------------------------------------------------------- split Fp12 (own half h)
// Own half of the product of two FULL Fp12 values a, b (both known to the lane): even lane c0 = a0 b0 + v a1 b1,
// odd lane c1 = a0 b1 + a1 b0.  Two Fp6 products per lane.
BLS_CALL __device__ void fp12h_mul_full(fp6& r, const fp12& a_in, const fp12& b_in, uint32_t m) {
  const fp12 a = a_in, b = b_in;
  const fp6 y1 = sel(m, b.c1, b.c0), y2 = sel(m, b.c0, b.c1);
  fp6 p1, p2, vp2;
  fp6_mul(p1, a.c0, y1);
  fp6_mul(p2, a.c1, y2);
  fp6_mul_v(vp2, p2);
  const fp6 q = sel(m, p2, vp2);
  fp6_add(r, p1, q);
}

// Own half of a*b for split a, b.
__device__ __forceinline__ void fp12h_mul_inl(fp6& r, const fp6& ah_in, const fp6& bh_in, uint32_t m) {
  const fp6 ah = ah_in, bh = bh_in;
  fp6 ao, bo;
  pair_swap(ao, ah);
  pair_swap(bo, bh);
  // even: (a0 b0) + v (a1 b1) with a0 = ah, a1 = ao; odd: (a0 b1) + (a1 b0) with a0 = ao, a1 = ah
  const fp6 x1 = sel(m, ao, ah), x2 = sel(m, ah, ao);
  fp6 p1, p2, vp2;
  fp6_mul(p1, x1, bh);
  fp6_mul(p2, x2, bo);
  fp6_mul_v(vp2, p2);
  const fp6 q = sel(m, p2, vp2);
  fp6_add(r, p1, q);
}
BLS_CALL __device__ void fp12h_mul(fp6& r, const fp6& ah_in, const fp6& bh_in, uint32_t m) { fp12h_mul_inl(r, ah_in, bh_in, m); }

// conj: c1 -> -c1 (odd lane negates)
__device__ __forceinline__ void fp12h_conj(fp6& r, const fp6& h, uint32_t m) {
  fp6 n;
  fp6_neg(n, h);
  r = sel(m, n, h);
}

// x -> x^(p^j): coefficient k = 2i + h (h = lane parity) of w^k is conj^j(c) * gamma_{j,k}
BLS_CALL __device__ void fp12h_frobenius(fp6& r, const fp6& h_in, int j, uint32_t m) {
  const fp6 h = h_in;
  const fp2* g = j == 1 ? FROB1 : (j == 2 ? FROB2 : FROB3);
  const fp2* src[3] = {&h.c0, &h.c1, &h.c2};
  fp2 out[3];
  for (int i = 0; i < 3; ++i) {
    fp2 c = *src[i];
    if (j & 1) fp2_conj(c, c);
    const fp2 gk = sel(m, g[2 * i + 1], g[2 * i]);
    fp2_mul(out[i], c, gk);
  }
  r.c0 = out[0];
  r.c1 = out[1];
  r.c2 = out[2];
}

// Granger-Scott cyclotomic squaring on the split value: five Fp2 squarings per lane (nine on one lane).
// Even lane holds (z0, z4, z3) = (c0.c0, c0.c1, c0.c2), odd lane (z2, z1, z5) = (c1.c0, c1.c1, c1.c2); the Fp4 pairs
// are (z0, z1), (z2, z3), (z4, z5).  The even lane squares pair (z0, z1) and z4, z4 + z5; the odd lane pair (z2, z3)
// and z5.  Outputs as fp12_cyclotomic_sqr: z0' = 3 t0 - 2 z0, z1' = 3 t1 + 2 z1, z2' = 3 xi t5 + 2 z2,
// z3' = 3 t4 - 2 z3, z4' = 3 t2 - 2 z4, z5' = 3 t3 + 2 z5.
BLS_CALL __device__ void fp12h_cyc_sqr(fp6& r, const fp6& h_in, uint32_t m) {
  const fp6 h = h_in;
  fp6 o;
  pair_swap(o, h);  // even: (z2, z1, z5); odd: (z0, z4, z3)
  const fp2 x = h.c0;                // even z0 | odd z2
  const fp2 y = sel(m, o.c2, o.c1);  // even z1 | odd z3
  const fp2 w = sel(m, h.c2, h.c1);  // even z4 | odd z5
  fp2 v, xy;
  fp2_add(v, h.c1, o.c2);            // even z4 + z5 (odd: unused)
  fp2_add(xy, x, y);
  fp2 S1, S2, S3, S4, S5;
  fp2_sqr(S1, x);
  fp2_sqr(S2, y);
  fp2_sqr(S3, xy);
  fp2_sqr(S4, w);
  fp2_sqr(S5, v);
  fp2 te, to, t;
  fp2_mul_xi(te, S2);
  fp2_add(te, te, S1);  // even t0 | odd t2
  fp2_sub(to, S3, S1);
  fp2_sub(to, to, S2);  // even t1 | odd t3
  fp2 S4o;
  pair_swap(S4o, S4);   // even z5^2 | odd z4^2
  fp2 t4, t5;
  fp2_mul_xi(t4, S4o);
  fp2_add(t4, t4, S4);  // even: t4 = z4^2 + xi z5^2
  fp2_sub(t5, S5, S4);
  fp2_sub(t5, t5, S4o);  // even: t5 = (z4 + z5)^2 - z4^2 - z5^2
  const fp2 p1 = sel(m, te, to);  // even sends t1, odd sends t2
  fp2 q1, q2;
  pair_swap(q1, p1);  // even receives t2 | odd receives t1
  pair_swap(q2, t5);  // odd receives t5
  fp2 xq2;
  fp2_mul_xi(xq2, q2);
  const fp2 u0 = sel(m, xq2, te), u1 = q1, u2 = sel(m, to, t4);
  fp6 nh;
  fp6_neg(nh, h);
  const fp6 zs = sel(m, h, nh);  // -z on the even lane, +z on the odd lane
  const fp2* us[3] = {&u0, &u1, &u2};
  const fp2* zz[3] = {&zs.c0, &zs.c1, &zs.c2};
  fp2 out[3];
  for (int k = 0; k < 3; ++k) {
    fp2 a;
    fp2_add(a, *us[k], *zz[k]);
    fp2_dbl(a, a);
    fp2_add(out[k], a, *us[k]);
  }
  r.c0 = out[0];
  r.c1 = out[1];
  r.c2 = out[2];
}

// Gathers the full value on both lanes.
__device__ __forceinline__ void fp12h_gather(fp12& full, const fp6& h, uint32_t m) {
  fp6 o;
  pair_swap(o, h);
  full.c0 = sel(m, o, h);
  full.c1 = sel(m, h, o);
}

// r = a^|x| for a in the cyclotomic subgroup (split)
BLS_CALL __device__ void fp12h_exp_xabs(fp6& r, const fp6& a_in, uint32_t m) {
  fp6 acc = a_in;  // the base stays in the caller's frame (see fp12_cyc_exp_xabs)
  for (int bit = 62; bit >= 0; --bit) {
    fp6 t;
    fp12h_cyc_sqr(t, acc, m);
    acc = t;
    if ((X_ABS >> bit) & 1ull) {  // through temporaries: acc's address is never taken
      fp6 x = acc, y;
      fp12h_mul(y, x, a_in, m);
      acc = y;
    }
  }
  r = acc;
}

// Karabina's compressed squarings on a lane pair (pairing.h fp12_cyc_exp_xabs_karabina).  Both lanes carry the same
// compressed state (z2..z5).  Per squaring the even lane squares z2, z3, z2 + z3 and the odd lane z4, z5, z4 + z5
// (three Fp2 squarings per lane instead of Granger-Scott's five), each forms A = 2 z z' and B = z^2 + xi z'^2 of its
// pair, the pair swaps (A, B), and both lanes form the new state:
//   z2' = 2 z2 + 3 xi (2 z4 z5),  z3' = 3 (z4^2 + xi z5^2) - 2 z3,  z4' = 3 (z2^2 + xi z3^2) - 2 z4,  z5' = 2 z5 + 3 (2 z2 z3).
// The state is bit-identical on both lanes, so every branch below is pair-uniform (DPP needs both lanes).
__device__ __forceinline__ void cyc_sqr_compressed_pair(cyc_c& c, uint32_t m) {
  const fp2 x = sel(m, c.z4, c.z2), y = sel(m, c.z5, c.z3);
  fp2 xy, sx, sy, sxy;
  fp2_add(xy, x, y);
  BLS_KAR_FP2_SQR(sx, x);
  BLS_KAR_FP2_SQR(sy, y);
  BLS_KAR_FP2_SQR(sxy, xy);
  fp2 A, B;
  fp2_sub(A, sxy, sx);
  fp2_sub(A, A, sy);  // even 2 z2 z3 | odd 2 z4 z5
  fp2_mul_xi(B, sy);
  fp2_add(B, B, sx);  // even z2^2 + xi z3^2 | odd z4^2 + xi z5^2
  fp2 Ao, Bo;
  pair_swap(Ao, A);
  pair_swap(Bo, B);
  const fp2 p45 = sel(m, A, Ao), q45 = sel(m, B, Bo);  // 2 z4 z5, z4^2 + xi z5^2
  const fp2 p23 = sel(m, Ao, A), q23 = sel(m, Bo, B);  // 2 z2 z3, z2^2 + xi z3^2
  fp2 t, v;
  fp2_mul_xi(t, p45);
  fp2_add(v, c.z2, t);
  fp2_add(v, v, v);
  fp2_add(c.z2, v, t);
  fp2_sub(v, q45, c.z3);
  fp2_add(v, v, v);
  fp2_add(c.z3, v, q45);
  fp2_sub(v, q23, c.z4);
  fp2_add(v, v, v);
  fp2_add(c.z4, v, q23);
  fp2_add(v, c.z5, p23);
  fp2_add(v, v, v);
  fp2_add(c.z5, v, p23);
}

#ifndef BLS_LG2_KAR_MUL
#define BLS_LG2_KAR_MUL fp12h_mul_inl  // inlined: n = 10,000 lane-pair Verify 27.82 -> 27.52 ms, C3 +0.9 %
#endif
// r = a^|x| (split) by compressed squarings; the six saved powers are decompressed on both lanes (one batch
// inversion) and multiplied as split values.  Degenerate inputs (a denominator 0) return true with r untouched, and
// fp12h_exp takes fp12h_exp_xabs from the caller's frame (off this function's stack depth).
BLS_CALL __device__ bool fp12h_exp_xabs_karabina(fp6& r, const fp6& a_in, uint32_t m) {
  static_assert(X_ABS == 0xd201000000010000ull, "the squaring counts below are |x|'s set bits");
  cyc_c c;
  {
    const fp6 h = a_in;
    fp6 o;
    pair_swap(o, h);  // even h = (z0, z4, z3), o = (z2, z1, z5); odd the other way round
    c.z2 = sel(m, h.c0, o.c0);
    c.z3 = sel(m, o.c2, h.c2);
    c.z4 = sel(m, o.c1, h.c1);
    c.z5 = sel(m, h.c2, o.c2);
  }
  cyc_c st[6];
  int s = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; ++k) {
    cyc_sqr_compressed_pair(c, m);
    if (k == 16 || k == 48 || k == 57 || k == 60 || k == 62 || k == 63) st[s++] = c;
  }
  // The six powers' z1 parts and decompressions are dealt out over the pair (even lane: powers 0, 2, 4; odd lane:
  // 1, 3, 5 -- three rounds instead of six); the batch inversion stays shared, and each lane hands its partner the
  // partner's half of the power it decompressed.  The back-substitution runs from power 5 down, so each round's two
  // inverses are ready just before its decompression, and only the running product stays live.
  fp2 nm[3], den[6];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    cyc_c cp;
    cp.z2 = sel(m, st[2 * k + 1].z2, st[2 * k].z2);
    cp.z3 = sel(m, st[2 * k + 1].z3, st[2 * k].z3);
    cp.z4 = sel(m, st[2 * k + 1].z4, st[2 * k].z4);
    cp.z5 = sel(m, st[2 * k + 1].z5, st[2 * k].z5);
    fp2 dm, o;
    cyc_z1_parts(nm[k], dm, cp);
    pair_swap_words<24>(&o.c0.v[0], &dm.c0.v[0]);
    den[2 * k] = sel(m, o, dm);
    den[2 * k + 1] = sel(m, dm, o);
  }
  fp2 pre[6];
  pre[0] = den[0];
#pragma unroll
  for (s = 1; s < 6; ++s) fp2_mul(pre[s], pre[s - 1], den[s]);
  if (fp2_is_zero(pre[5])) return true;  // same on both lanes
  fp2 inv;
  fp2_inv(inv, pre[5]);
  fp6 acc;
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    fp2 is_odd, is_even;  // 1 / den[2k + 1], 1 / den[2k]
    fp2_mul(is_odd, inv, pre[2 * k]);
    fp2_mul(inv, inv, den[2 * k + 1]);
    if (k > 0) {
      fp2_mul(is_even, inv, pre[2 * k - 1]);
      fp2_mul(inv, inv, den[2 * k]);
    } else {
      is_even = inv;
    }
    cyc_c cp;
    cp.z2 = sel(m, st[2 * k + 1].z2, st[2 * k].z2);
    cp.z3 = sel(m, st[2 * k + 1].z3, st[2 * k].z3);
    cp.z4 = sel(m, st[2 * k + 1].z4, st[2 * k].z4);
    cp.z5 = sel(m, st[2 * k + 1].z5, st[2 * k].z5);
    fp2 z1;
    fp2_mul(z1, nm[k], sel(m, is_odd, is_even));
    fp12 d;
    cyc_decompress(d, cp, z1);
    const fp6 own = sel(m, d.c1, d.c0), theirs = sel(m, d.c0, d.c1);
    fp6 got;
    pair_swap(got, theirs);
    const fp6 h_odd = sel(m, own, got), h_even = sel(m, got, own);  // this lane's halves of d_{2k+1}, d_{2k}
    if (k == 2) {
      acc = h_odd;
    } else {
      fp6 x = acc, y;
      BLS_LG2_KAR_MUL(y, x, h_odd, m);
      acc = y;
    }
    fp6 x = acc, y;
    BLS_LG2_KAR_MUL(y, x, h_even, m);
    acc = y;
  }
  r = acc;
  return false;
}

#ifndef BLS_LG2_KARABINA
#define BLS_LG2_KARABINA 1
#endif
__device__ __forceinline__ void fp12h_exp(fp6& r, const fp6& a_in, uint32_t m) {
#if BLS_LG2_KARABINA
  if (fp12h_exp_xabs_karabina(r, a_in, m)) fp12h_exp_xabs(r, a_in, m);
#else
  fp12h_exp_xabs(r, a_in, m);
#endif
}

// final_exponentiation (pairing.h) on a split value: same formula, split operations; the products inlined (as the
// quad's fp12q_mul: a call sends its operands through the stack).
BLS_CALL __device__ void final_exponentiation_split(fp6& r, const fp6& f_in, uint32_t m) {
  // temporaries scoped so their frame slots can be shared (pairing_lds.h final_exponentiation_l); r may alias f_in
  fp6 mm;
  {  // easy part: f^((p^6-1)(p^2+1)); the inverse is computed on both lanes from the gathered value
    fp6 t;
    fp6 fi;
    {
      fp12 full, inv;
      fp12h_gather(full, f_in, m);
      fp12_inv(inv, full);
      fi = sel(m, inv.c1, inv.c0);
    }
    fp12h_conj(t, f_in, m);
    fp12h_mul_inl(mm, t, fi, m);
    fp12h_frobenius(t, mm, 2, m);
    fp12h_mul_inl(mm, t, mm, m);
  }
  // hard part
  fp6 t1;
  {
    fp6 t0, u;
    fp12h_exp(t0, mm, m);
    fp12h_mul_inl(t0, t0, mm, m);
    fp12h_conj(t0, t0, m);
    fp12h_exp(u, t0, m);
    fp12h_mul_inl(u, u, t0, m);
    fp12h_conj(t0, u, m);
    fp12h_exp(u, t0, m);
    fp12h_conj(u, u, m);
    fp12h_frobenius(t1, t0, 1, m);
    fp12h_mul_inl(t1, t1, u, m);
  }
  fp6 t2;
  {
    fp6 u;
    fp12h_exp(u, t1, m);
    fp12h_exp(u, u, m);
    fp12h_frobenius(t2, t1, 2, m);
    fp12h_mul_inl(t2, t2, u, m);
    fp12h_conj(u, t1, m);
    fp12h_mul_inl(t2, t2, u, m);
  }
  {
    fp6 u;
    fp12h_cyc_sqr(u, mm, m);
    fp12h_mul_inl(u, u, mm, m);
    fp12h_mul_inl(r, t2, u, m);
  }
}

// Is the split value 1?  Even half must be (1, 0, 0), odd half 0; both lanes get the answer.
__device__ __forceinline__ bool fp12h_is_one(const fp6& h, uint32_t m) {
  fp6 one6;
  fp6_set_one(one6);
  fp6 zero6;
  fp6_set_zero(zero6);
  const fp6 want = sel(m, zero6, one6);
  uint32_t acc = 0;
  const uint32_t* a = &h.c0.c0.v[0];
  const uint32_t* b = &want.c0.c0.v[0];
  for (int i = 0; i < 72; ++i) acc |= a[i] ^ b[i];
  const uint32_t mine = acc == 0 ? 1u : 0u;
  return (mine & pair_swap(mine)) != 0;
}

// Pairing-product check over n pairs split across a lane pair: this lane takes pairs i with i % 2 == parity
// (at most MAXN of them).  Both lanes must call it together with the same n.  Returns prod e(P_i, Q_i) == 1 on
// both lanes.  P_i / Q_i are read through callables so the caller decides where the pairs come from.
// Both lanes hold a full Fp12 (their own Miller value): the check prod == 1 after the split final exponentiation.
static __device__ bool lg2_finish(const fp12& f, uint32_t m) {
  fp12 g;
  fp12 mine = f;
  // combine the two lanes' Miller values: own half of f_even * f_odd
  pair_swap(g.c0, mine.c0);
  pair_swap(g.c1, mine.c1);
  fp12 fe, fo;
  fe.c0 = sel(m, g.c0, mine.c0);
  fe.c1 = sel(m, g.c1, mine.c1);
  fo.c0 = sel(m, mine.c0, g.c0);
  fo.c1 = sel(m, mine.c1, g.c1);
  fp6 h, e;
  fp12h_mul_full(h, fe, fo, m);
  final_exponentiation_split(e, h, m);
  return fp12h_is_one(e, m);
}

// ---------------------------------------------------------------- one Miller loop split across a lane pair
// f_{|x|, Q}(P) (miller_loop_multi<1>: the same steps, the same f) held split as above (even lane c0, odd lane c1).
// Both lanes carry the same T and run the same doubling/addition steps (the point arithmetic and its lines are
// computed redundantly); the Fp12 work, which is 3/4 of a step, is split:
//   * squaring: f = a + b w, f^2 = ((a + b)(a + v b) - t - v t) + 2 t w with t = a b: the even lane forms the first
//     product, the odd lane t, one exchange brings t to the even lane -- one Fp6 product per lane instead of two;
//   * line: l = (g0 + g1 v) + (h1 v) w, f l = (a L0 + v b L1) + (a L1 + b L0) w: the even lane computes a L0 and
//     b L1, the odd lane b L0 and a L1 (5 + 3 Fp2 products per lane instead of 13).
// A step costs ~55 products of latency instead of 100.  Both lanes must call it together with the same P, Q.
__device__ __forceinline__ void fp12h_sqr_split(fp6& h, uint32_t m) {
  fp6 o;
  pair_swap(o, h);
  const fp6 a = sel(m, o, h), b = sel(m, h, o);
  fp6 s0, vb, s1;
  fp6_add(s0, a, b);
  fp6_mul_v(vb, b);
  fp6_add(s1, a, vb);
  const fp6 x = sel(m, a, s0), y = sel(m, b, s1);  // odd: a b | even: (a + b)(a + v b)
  fp6 p;
  LG2_FP6_MUL(p, x, y);
  fp6 t;
  pair_swap(t, p);  // even receives t = a b
  fp6 vt, c0, c1;
  fp6_mul_v(vt, t);
  fp6_sub(c0, p, t);
  fp6_sub(c0, c0, vt);
  fp6_add(c1, p, p);
  h = sel(m, c1, c0);
}
__device__ __forceinline__ void fp12h_mul_line_split(fp6& h, const fp2& g0, const fp2& g1, const fp2& h1, uint32_t m) {
  fp6 o;
  pair_swap(o, h);
  const fp6 a = sel(m, o, h), b = sel(m, h, o);
  const fp6 x = sel(m, b, a), y = sel(m, a, b);
  fp6 t0, t1, vt1, r;
  fp6_mul_01(t0, x, g0, g1);  // even a L0 | odd b L0
  fp6_mul_1(t1, y, h1);       // even b h1 v | odd a h1 v
  fp6_mul_v(vt1, t1);
  fp6_add(r, t0, sel(m, t1, vt1));
  h = r;
}
// pairing.h miller_dbl_step_inl split across the pair: the same formulas and the same (canonical) outputs on both
// lanes, with the Fp2 products dealt out in three uniform slots per phase (even | odd):
//   phase 1: Y^2 | X^2,  Z Z | X Y,  (Y + Z)^2 on both                -> swap (B, C) for (J, XY)
//   phase 2: G G | A (B - F),  E E | B H,  H y_P | 3J x_P            -> swap (Y3, h1) for (X3, Z3, g1)
// 15 products of latency instead of 25.
__device__ __forceinline__ fp sel(uint32_t m, const fp& if_odd, const fp& if_even) {
  fp r;
  sel_words<12>(&r.v[0], m, &if_odd.v[0], &if_even.v[0]);
  return r;
}
__device__ __forceinline__ void miller_dbl_step_split(g2j& T, fp2& g0, fp2& g1, fp2& h1, const fp& xp, const fp& yp,
                                                      uint32_t m) {
  fp2 r1, r2, r3, s;
  fp2_sqr(r1, sel(m, T.x, T.y));                     // even B = Y^2 | odd J = X^2
  fp2_mul(r2, sel(m, T.x, T.z), sel(m, T.y, T.z));   // even C = Z^2 | odd X Y
  fp2_add(s, T.y, T.z);
  fp2_sqr(r3, s);                                    // D = (Y + Z)^2 on both lanes
  fp2 o1, o2;
  pair_swap(o1, r1);
  pair_swap(o2, r2);
  const fp2 B = sel(m, o1, r1), J = sel(m, r1, o1), C = sel(m, o2, r2), XY = sel(m, r2, o2), D = r3;
  fp2 A, E, F, G, H, t;
  fp2_half(A, XY);
  fp2_mul_3b2(E, C);
  fp2_add(F, E, E);
  fp2_add(F, F, E);
  fp2_add(G, B, F);
  fp2_half(G, G);
  fp2_sub(H, D, B);
  fp2_sub(H, H, C);
  fp2_sub(g0, E, B);
  fp2 J3, BF;
  fp2_add(J3, J, J);
  fp2_add(J3, J3, J);
  fp2_sub(BF, B, F);
  fp2 p1, p2, p3;
  fp2_mul(p1, sel(m, A, G), sel(m, BF, G));          // even G^2 | odd X3 = A (B - F)
  fp2_mul(p2, sel(m, B, E), sel(m, H, E));           // even E^2 | odd Z3 = B H
  fp2_mul_fp(p3, sel(m, J3, H), sel(m, xp, yp));     // even H y_P | odd g1 = 3J x_P
  fp2 Y3, E3, hneg;
  fp2_add(E3, p2, p2);
  fp2_add(E3, E3, p2);
  fp2_sub(Y3, p1, E3);                               // even: G^2 - 3 E^2
  fp2_neg(hneg, p3);                                 // even: h1 = -H y_P
  const fp2 s1 = sel(m, p1, Y3), s2 = sel(m, p2, hneg), s3 = sel(m, p3, hneg);
  fp2 q1, q2, q3;
  pair_swap(q1, s1);  // even receives X3 | odd receives Y3
  pair_swap(q2, s2);  // even receives Z3 | odd receives h1
  pair_swap(q3, s3);  // even receives g1
  T.x = sel(m, p1, q1);
  T.y = sel(m, q1, Y3);
  T.z = sel(m, p2, q2);
  g1 = sel(m, p3, q3);
  h1 = sel(m, q2, hneg);
}

#ifndef BLS_LQ4_DBL_SPLIT
#define BLS_LQ4_DBL_SPLIT 1
#endif
BLS_CALL __device__ void miller_loop_split(fp6& h_out, const g1a& P_in, const g2a& Q_in, uint32_t m,
                                           g2j* T_out = nullptr) {
  const g1a P = P_in;
  const g2a Q = Q_in;
  g2j T;
  T.x = Q.x;
  T.y = Q.y;
  fp2_set_one(T.z);
  fp6 one6, zero6, h;
  fp6_set_one(one6);
  fp6_set_zero(zero6);
  h = sel(m, zero6, one6);
  for (int bit = 62; bit >= 0; --bit) {
    if ((bit & 7) == 7) BLS_RACE_POLL();
    if (bit != 62) fp12h_sqr_split(h, m);
    fp2 g0, g1, h1;
#if BLS_LQ4_DBL_SPLIT
    miller_dbl_step_split(T, g0, g1, h1, P.x, P.y, m);
#else
    miller_dbl_step_inl(T, g0, g1, h1, P.x, P.y);
#endif
    fp12h_mul_line_split(h, g0, g1, h1, m);
    if ((X_ABS >> bit) & 1ull) {
      miller_add_step_inl(T, g0, g1, h1, Q, P.x, P.y);
      fp12h_mul_line_split(h, g0, g1, h1, m);
    }
  }
  fp12h_conj(h_out, h, m);
  if (T_out) *T_out = T;
}

// Partner lane across the two pairs of a quad (lane ^ 2).  All four lanes must be active.
__device__ __forceinline__ uint32_t quad_swap(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E /* quad_perm [2,3,0,1] */, 0xF, 0xF, false);
#else
  return v;
#endif
}

// ---------------------------------------------------------------- the final exponentiation on a lane quad
// The value is held in full on all four lanes (bit-identical), and the work of each step is dealt out:
//   * Fp12 product: lane q computes one of the four Fp6 products of the schoolbook form (a0 b0, a1 b1, a0 b1, a1 b0),
//     the pairs combine theirs into c0 = a0 b0 + v a1 b1 (lanes 0, 1) and c1 = a0 b1 + a1 b0 (lanes 2, 3), and one
//     exchange across the pairs gives every lane both halves: one Fp6 product per lane instead of two on a pair;
//   * Karabina's compressed squaring: its six Fp2 squarings as two rounds of four (z2 | z3 | z4 | z5, then
//     z2 + z3 | z4 + z5 on lanes 0, 1): two squarings of latency instead of three; then each lane forms one of the
//     four new coordinates and the quad broadcasts them (half the additions per lane).
// Everything else (decompression, the easy part's inversion, Frobenius maps) runs redundantly on all lanes on the
// same data, so every branch is quad-uniform (DPP needs all four lanes).
template <int SRC>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, SRC * 0x55 /* quad_perm [SRC,SRC,SRC,SRC] */, 0xF, 0xF, false);
#else
  return v;
#endif
}
template <int SRC>
__device__ __forceinline__ fp2 quad_bcast(const fp2& s) {
  fp2 d;
#pragma unroll
  for (int i = 0; i < 24; ++i) (&d.c0.v[0])[i] = quad_bcast<SRC>((&s.c0.v[0])[i]);
  return d;
}
__device__ __forceinline__ void quad_swap(fp6& d, const fp6& s) {
#pragma unroll
  for (int i = 0; i < 72; ++i) (&d.c0.c0.v[0])[i] = quad_swap((&s.c0.c0.v[0])[i]);
}
struct quad_m {  // lane masks within the quad (q = lane & 3)
  uint32_t odd, hi, cross;  // q & 1, q >= 2, q in {1, 2}
  __device__ explicit quad_m(int q)
      : odd((q & 1) ? ~0u : 0u), hi((q & 2) ? ~0u : 0u), cross(((q ^ (q >> 1)) & 1) ? ~0u : 0u) {}
};

// Inlined into its callers: as a call, its two 576-byte operands and result go through the stack around every product
// (profiles/r04/oct_probe*.txt: fp12q_mul 55.8k -> 41.3k cycles, the quad final exponentiation 13.3M -> 10.2M).
#ifndef BLS_FP12Q_MUL_ATTR
#define BLS_FP12Q_MUL_ATTR static __forceinline__
#endif
BLS_FP12Q_MUL_ATTR __device__ void fp12q_mul(fp12& r, const fp12& a_in, const fp12& b_in, const quad_m& qm) {
  const fp12 a = a_in, b = b_in;
  const fp6 x = sel(qm.odd, a.c1, a.c0);    // a0 | a1 | a0 | a1
  const fp6 y = sel(qm.cross, b.c1, b.c0);  // b0 | b1 | b1 | b0
  fp6 p, o, vp, vo, t0, t1, t2;
  LG2_FP6_MUL(p, x, y);
  pair_swap(o, p);
  fp6_mul_v(vp, p);
  fp6_mul_v(vo, o);
  fp6_add(t0, p, vo);  // lane 0: a0 b0 + v a1 b1
  fp6_add(t1, o, vp);  // lane 1: the same sum
  fp6_add(t2, p, o);   // lanes 2, 3: a0 b1 + a1 b0
  const fp6 mine = sel(qm.hi, t2, sel(qm.odd, t1, t0));
  fp6 other;
  quad_swap(other, mine);
  r.c0 = sel(qm.hi, other, mine);
  r.c1 = sel(qm.hi, mine, other);
}

// Arbitrary permutation within each quad: lane i takes lane CTRL's 2-bit field i (quad_perm [p0, p1, p2, p3]).
template <int CTRL>
__device__ __forceinline__ fp2 quad_perm(const fp2& s) {
  fp2 d;
#pragma unroll
  for (int i = 0; i < 24; ++i)
    (&d.c0.v[0])[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(&s.c0.v[0])[i], CTRL, 0xF, 0xF, false);
  return d;
}

// The six Fp2 squarings as two rounds of four, then each lane forms ONE new coordinate (z2' | z3' | z4' | z5') from the
// squares it needs (three DPP permutations bring them) and the quad broadcasts the four: the additions after the
// squarings are ~11 Fp2 operations per lane instead of every lane forming all four coordinates (22).
//   lane 0: z2' = 2 z2 + 3 xi ((z4 + z5)^2 - z4^2 - z5^2)     lane 1: z3' = 3 (z4^2 + xi z5^2) - 2 z3
//   lane 2: z4' = 3 (z2^2 + xi z3^2) - 2 z4                    lane 3: z5' = 2 z5 + 3 ((z2 + z3)^2 - z2^2 - z3^2)
__device__ __forceinline__ void cyc_sqr_compressed_quad(cyc_c& c, const quad_m& qm) {
  // round 1: z2 | z3 | z4 | z5 (also this lane's own coordinate)
  const fp2 xa = sel(qm.hi, sel(qm.odd, c.z5, c.z4), sel(qm.odd, c.z3, c.z2));
  // round 2: z2 + z3 | z4 + z5 (lanes 2, 3 repeat lanes 0, 1)
  fp2 s23, s45;  // canonical: the squaring routine forms a0 + p - a1
  fp2_add(s23, c.z2, c.z3);
  fp2_add(s45, c.z4, c.z5);
  const fp2 xb = sel(qm.odd, s45, s23);
  fp2 ra, rb;
#if BLS_HEX
  // both rounds at once: the low half squares xa, the high half xb; one exchange gives each half the other's
  {
    const uint32_t h = hx_mask();
    fp2 r;
    BLS_KAR_FP2_SQR(r, sel(h, xb, xa));
    const fp2 o = hx_xchg(r);
    ra = sel(h, o, r);
    rb = sel(h, r, o);
  }
#else
  BLS_KAR_FP2_SQR(ra, xa);
  BLS_KAR_FP2_SQR(rb, xb);
#endif
  const fp2 X = quad_perm<0x0A>(ra);  // [2, 2, 0, 0]: z4^2 | z4^2 | z2^2 | z2^2
  const fp2 Y = quad_perm<0x5F>(ra);  // [3, 3, 1, 1]: z5^2 | z5^2 | z3^2 | z3^2
  const fp2 W = quad_perm<0x05>(rb);  // [1, 1, 0, 0]: (z4 + z5)^2 on lane 0, (z2 + z3)^2 on lane 3
  fp2 A, B, xiA, xiY, zz, nzz, V3, out;
  fp2_sub(A, W, X);
  fp2_sub(A, A, Y);  // 2 z4 z5 (lane 0) | 2 z2 z3 (lane 3)
  fp2_mul_xi(xiY, Y);
  fp2_add(B, xiY, X);  // z4^2 + xi z5^2 (lane 1) | z2^2 + xi z3^2 (lane 2)
  fp2_mul_xi(xiA, A);
  const fp2 V = sel(qm.cross, B, sel(qm.odd, A, xiA));
  fp2_add(V3, V, V);
  fp2_add(V3, V3, V);
  fp2_add(zz, xa, xa);
  fp2_neg(nzz, zz);
  fp2_add(out, V3, sel(qm.cross, nzz, zz));  // 3 V + 2 z (lanes 0, 3) | 3 V - 2 z (lanes 1, 2)
  c.z2 = quad_bcast<0>(out);
  c.z3 = quad_bcast<1>(out);
  c.z4 = quad_bcast<2>(out);
  c.z5 = quad_bcast<3>(out);
}

template <int SRC>
__device__ __forceinline__ void quad_bcast12(fp12& d, const fp12& s) {
#pragma unroll
  for (int i = 0; i < 144; ++i) (&d.c0.c0.c0.v[0])[i] = quad_bcast<SRC>((&s.c0.c0.c0.v[0])[i]);
}
__device__ __forceinline__ void cyc_sel(cyc_c& r, uint32_t m, const cyc_c& if_set, const cyc_c& if_clear) {
  r.z2 = sel(m, if_set.z2, if_clear.z2);
  r.z3 = sel(m, if_set.z3, if_clear.z3);
  r.z4 = sel(m, if_set.z4, if_clear.z4);
  r.z5 = sel(m, if_set.z5, if_clear.z5);
}

// r = a^|x| on a quad (a in the cyclotomic subgroup, in full on every lane), pairing.h fp12_cyc_exp_xabs_karabina's
// steps; the degenerate case (a saved power with z2 = z3 = 0) takes the one-lane Granger-Scott exponentiation on
// every lane.
// Returns true, r untouched, in the degenerate case (fp12q_exp_xabs then takes Granger-Scott from the caller's frame,
// keeping that chain off this function's stack depth).
BLS_CALL __device__ bool fp12q_exp_xabs_karabina(fp12& r, const fp12& a_in, const quad_m& qm) {
  static_assert(X_ABS == 0xd201000000010000ull, "the squaring counts below are |x|'s set bits");
  cyc_c c;
  c.z2 = a_in.c1.c0;
  c.z3 = a_in.c0.c2;
  c.z4 = a_in.c0.c1;
  c.z5 = a_in.c1.c2;
  cyc_c st[6];
  int s = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; ++k) {
    if ((k & 7) == 0) BLS_RACE_POLL();
    cyc_sqr_compressed_quad(c, qm);
    if (k == 16 || k == 48 || k == 57 || k == 60 || k == 62 || k == 63) st[s++] = c;
  }
  // The six powers' z1 parts and decompressions are dealt out over the quad (lane q takes powers q and, on lanes 0
  // and 1, q + 4: two rounds instead of six), then broadcast; the batch inversion and the products stay shared.
  cyc_c cA, cB;
  cyc_sel(cA, qm.odd, st[1], st[0]);
  {
    cyc_c hi;
    cyc_sel(hi, qm.odd, st[3], st[2]);
    cyc_sel(cA, qm.hi, hi, cA);
  }
  cyc_sel(cB, qm.odd, st[5], st[4]);
  fp2 nA, dA, nB, dB;
  cyc_z1_parts(nA, dA, cA);
  cyc_z1_parts(nB, dB, cB);
  const fp2 den[6] = {quad_bcast<0>(dA), quad_bcast<1>(dA), quad_bcast<2>(dA), quad_bcast<3>(dA), quad_bcast<0>(dB),
                      quad_bcast<1>(dB)};
  fp2 pre[6];
  pre[0] = den[0];
#pragma unroll
  for (s = 1; s < 6; ++s) fp2_mul(pre[s], pre[s - 1], den[s]);
  if (fp2_is_zero(pre[5])) return true;  // the same on all four lanes
  fp2 inv;
  fp2_inv(inv, pre[5]);
  BLS_RACE_POLL();
  fp2 is[6];  // 1 / den[s] by back-substitution
#pragma unroll
  for (s = 5; s > 0; --s) {
    fp2_mul(is[s], inv, pre[s - 1]);
    fp2_mul(inv, inv, den[s]);
  }
  is[0] = inv;
  fp2 z1A, z1B;
  fp2_mul(z1A, nA, sel(qm.hi, sel(qm.odd, is[3], is[2]), sel(qm.odd, is[1], is[0])));
  fp2_mul(z1B, nB, sel(qm.odd, is[5], is[4]));
  fp12 xA, xB;
  cyc_decompress(xA, cA, z1A);
  cyc_decompress(xB, cB, z1B);
  // acc = d5 d4 d3 d2 d1 d0 (pairing.h's order)
  fp12 acc, d;
  quad_bcast12<1>(acc, xB);
  quad_bcast12<0>(d, xB);
  {
    fp12 x = acc;
    fp12q_mul(acc, x, d, qm);
  }
  quad_bcast12<3>(d, xA);
  {
    fp12 x = acc;
    fp12q_mul(acc, x, d, qm);
  }
  BLS_RACE_POLL();
  quad_bcast12<2>(d, xA);
  {
    fp12 x = acc;
    fp12q_mul(acc, x, d, qm);
  }
  quad_bcast12<1>(d, xA);
  {
    fp12 x = acc;
    fp12q_mul(acc, x, d, qm);
  }
  BLS_RACE_POLL();
  quad_bcast12<0>(d, xA);
  {
    fp12 x = acc;
    fp12q_mul(acc, x, d, qm);
  }
  r = acc;
  return false;
}
BLS_HD BLS_INLINE void fp12q_exp_xabs(fp12& r, const fp12& a_in, const quad_m& qm) {
  if (fp12q_exp_xabs_karabina(r, a_in, qm)) fp12_cyc_exp_xabs_gs(r, a_in);
}

// final_exponentiation (pairing.h) on a quad: the same formula and the same result on every lane.
BLS_CALL __device__ void final_exponentiation_quad(fp12& r, const fp12& f_in, const quad_m& qm) {
  BLS_RACE_POLL();
  // temporaries scoped so their frame slots can be shared (pairing_lds.h final_exponentiation_l); r may alias f_in
  fp12 m;
  {
    fp12 t, fi;
    fp12_conj(t, f_in);
    fp12_inv(fi, f_in);
    fp12q_mul(m, t, fi, qm);
    fp12_frobenius(t, m, 2);
    fp12q_mul(m, t, m, qm);
  }
  fp12 t1;
  {
    fp12 t0, u;
    fp12q_exp_xabs(t0, m, qm);
    fp12q_mul(t0, t0, m, qm);
    fp12_conj(t0, t0);
    fp12q_exp_xabs(u, t0, qm);
    fp12q_mul(u, u, t0, qm);
    fp12_conj(t0, u);
    fp12q_exp_xabs(u, t0, qm);
    fp12_conj(u, u);
    fp12_frobenius(t1, t0, 1);
    fp12q_mul(t1, t1, u, qm);
  }
  BLS_RACE_POLL();
  fp12 t2;
  {
    fp12 u;
    fp12q_exp_xabs(u, t1, qm);
    fp12q_exp_xabs(u, u, qm);
    fp12_frobenius(t2, t1, 2);
    fp12q_mul(t2, t2, u, qm);
    fp12_conj(u, t1);
    fp12q_mul(t2, t2, u, qm);
  }
  BLS_RACE_POLL();
  {
    fp12 u;
    fp12_cyclotomic_sqr(u, m);
    fp12q_mul(u, u, m, qm);
    fp12q_mul(r, t2, u, qm);
  }
}

#ifndef BLS_LQ4_FE_QUAD
#define BLS_LQ4_FE_QUAD 1
#endif

// ---------------------------------------------------------------- one Miller accumulator for both pairs (round 5)
// lq4_verify's two Miller loops share ONE accumulator held in full on the quad: f <- f^2 lA lB, where each pair's
// doubling / addition step leaves its line on both of its lanes (miller_dbl_step_split, miller_add_step_inl) and one
// exchange across the pairs gives every lane both lines.  Per bit: the two doubling steps side by side on the pairs
// (as before), the Fp12 squaring as two Fp6 products with their Fp2 products split over a pair (fp12q_sqr), the
// product of the two lines (eight Fp2 products in two slots over the quad) and one quad Fp12 product (fp12q_mul)
// -- instead of each pair squaring its own split value and multiplying it by its own line.  f_A f_B is the same
// element either way (the squarings distribute over the product), so the final exponentiation's input and every
// status are unchanged.  BLS_LQ4_SHARED=0 builds the two split loops.  Measured (profiles/r05/lq4_shared_ab.json):
// sigagg's quad check (the main translation unit) gains, C3 489k -> 501k aggregates/s with one call in flight and
// 589k -> 606k on two streams; the split-Fp2 builds (octet and sixteen-lane n = 1 checks) lose (check 6.41 -> 6.57
// ms: there the split loop's Fp12 squaring is already shared by the twin halves), so they keep the split loops.
#ifndef BLS_LQ4_SHARED
#if BLS_FP2_PAIR
#define BLS_LQ4_SHARED 0
#else
#define BLS_LQ4_SHARED 1
#endif
#endif
#if BLS_LQ4_SHARED
// tower.h fp6_mul (Karatsuba) with its six Fp2 products dealt over a lane pair: the even lane forms a0 b0, a1 b1,
// a2 b2, the odd lane (a1 + a2)(b1 + b2), (a0 + a1)(b0 + b1), (a0 + a2)(b0 + b2); one exchange; both combine them as
// fp6_mul does.  Both lanes of the pair must be active and hold the same operands.
__device__ __forceinline__ void fp6_mul_pair(fp6& r, const fp6& a_in, const fp6& b_in, uint32_t odd) {
  const fp6 a = a_in, b = b_in;
  fp2 s0, s1, p0, p1, p2;
  fp2_add_lazy(s0, a.c1, a.c2);
  fp2_add_lazy(s1, b.c1, b.c2);
  fp2_mul(p0, sel(odd, s0, a.c0), sel(odd, s1, b.c0));
  fp2_add_lazy(s0, a.c0, a.c1);
  fp2_add_lazy(s1, b.c0, b.c1);
  fp2_mul(p1, sel(odd, s0, a.c1), sel(odd, s1, b.c1));
  fp2_add_lazy(s0, a.c0, a.c2);
  fp2_add_lazy(s1, b.c0, b.c2);
  fp2_mul(p2, sel(odd, s0, a.c2), sel(odd, s1, b.c2));
  fp2 o0, o1, o2;
  pair_swap(o0, p0);
  pair_swap(o1, p1);
  pair_swap(o2, p2);
  const fp2 t0 = sel(odd, o0, p0), t1 = sel(odd, o1, p1), t2 = sel(odd, o2, p2);
  const fp2 m12 = sel(odd, p0, o0), m01 = sel(odd, p1, o1), m02 = sel(odd, p2, o2);
  fp2 u0, u1, u2, x2;
  fp2_sub(u0, m12, t1);
  fp2_sub(u0, u0, t2);
  fp2_mul_xi(u0, u0);
  fp2_add(u0, u0, t0);
  fp2_sub(u1, m01, t0);
  fp2_sub(u1, u1, t1);
  fp2_mul_xi(x2, t2);
  fp2_add(u1, u1, x2);
  fp2_sub(u2, m02, t0);
  fp2_sub(u2, u2, t2);
  fp2_add(u2, u2, t1);
  r.c0 = u0;
  r.c1 = u1;
  r.c2 = u2;
}
// f = f^2 for f in full on the quad: X = (a + b)(a + v b) on lanes 0, 1 and Y = a b on lanes 2, 3, each split over its
// pair, one exchange across the pairs, then f^2 = (X - Y - v Y) + 2 Y w (fp12h_sqr_split's formula).
__device__ __forceinline__ void fp12q_sqr(fp12& f, const quad_m& qm) {
  const fp6 a = f.c0, b = f.c1;
  fp6 s0, vb, s1;
  fp6_add(s0, a, b);
  fp6_mul_v(vb, b);
  fp6_add(s1, a, vb);
  const fp6 x = sel(qm.hi, a, s0), y = sel(qm.hi, b, s1);
  fp6 p, o;
  fp6_mul_pair(p, x, y, qm.odd);
  quad_swap(o, p);
  const fp6 X = sel(qm.hi, o, p), Y = sel(qm.hi, p, o);
  fp6 vY, c0;
  fp6_mul_v(vY, Y);
  fp6_sub(c0, X, Y);
  fp6_sub(c0, c0, vY);
  fp6_add(f.c1, Y, Y);
  f.c0 = c0;
}
// f = f lA lB (f = lA lB when `first`): this pair's line (g0, g1, h1) on both of its lanes, the other pair's by one
// exchange; M = lA lB = (a0 b0 + xi ah bh, a0 b1 + a1 b0, a1 b1) + (0, a0 bh + ah b0, a1 bh + ah b1) w for
// l = (g0 + g1 v) + (h1 v) w, its eight Fp2 products as two slots over the quad.
__device__ __forceinline__ void fp12q_mul_two_lines(fp12& f, bool first, const fp2& g0, const fp2& g1, const fp2& h1,
                                                    const quad_m& qm) {
  fp2 og0, og1, oh1;
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    (&og0.c0.v[0])[i] = quad_swap((&g0.c0.v[0])[i]);
    (&og1.c0.v[0])[i] = quad_swap((&g1.c0.v[0])[i]);
    (&oh1.c0.v[0])[i] = quad_swap((&h1.c0.v[0])[i]);
  }
  const fp2 a0 = sel(qm.hi, og0, g0), a1 = sel(qm.hi, og1, g1), ah = sel(qm.hi, oh1, h1);  // pair A's line
  const fp2 b0 = sel(qm.hi, g0, og0), b1 = sel(qm.hi, g1, og1), bh = sel(qm.hi, h1, oh1);  // pair B's line
  fp2 sa, sb, x, y, o1, o2;
  fp2_add_lazy(sa, a0, a1);
  fp2_add_lazy(sb, b0, b1);
  x = sel(qm.hi, sel(qm.odd, ah, sa), sel(qm.odd, a1, a0));  // a0 b0 | a1 b1 | (a0 + a1)(b0 + b1) | ah bh
  y = sel(qm.hi, sel(qm.odd, bh, sb), sel(qm.odd, b1, b0));
  fp2_mul(o1, x, y);
  x = sel(qm.hi, sel(qm.odd, ah, a1), sel(qm.odd, ah, a0));  // a0 bh | ah b0 | a1 bh | ah b1
  y = sel(qm.hi, sel(qm.odd, b1, bh), sel(qm.odd, b0, bh));
  fp2_mul(o2, x, y);
  const fp2 p00 = quad_bcast<0>(o1), p11 = quad_bcast<1>(o1), s01 = quad_bcast<2>(o1), phh = quad_bcast<3>(o1);
  const fp2 q0 = quad_bcast<0>(o2), q1 = quad_bcast<1>(o2), q2 = quad_bcast<2>(o2), q3 = quad_bcast<3>(o2);
  fp12 M;
  fp2 t;
  fp2_mul_xi(t, phh);
  fp2_add(M.c0.c0, p00, t);
  fp2_sub(t, s01, p00);
  fp2_sub(M.c0.c1, t, p11);
  M.c0.c2 = p11;
  fp2_set_zero(M.c1.c0);
  fp2_add(M.c1.c1, q0, q1);
  fp2_add(M.c1.c2, q2, q3);
  if (first) {
    f = M;
  } else {
    fp12 x12 = f;
    fp12q_mul(f, x12, M, qm);
  }
}
// f_{|x|,Q_A}(P_A) f_{|x|,Q_B}(P_B), conjugated (x < 0), in full on every lane of the quad; lanes 0, 1 carry pair A's
// (P, Q) and T, lanes 2, 3 pair B's.  T_out: this pair's final T (pair B's gives the signature's G2 membership).
BLS_CALL __device__ void miller_loop_shared_quad(fp12& f_out, const g1a& P_in, const g2a& Q_in, const quad_m& qm,
                                                 uint32_t m, g2j* T_out) {
  const g1a P = P_in;
  const g2a Q = Q_in;
  g2j T;
  T.x = Q.x;
  T.y = Q.y;
  fp2_set_one(T.z);
  fp12 f;
  for (int bit = 62; bit >= 0; --bit) {
    if ((bit & 7) == 7) BLS_RACE_POLL();
    if (bit != 62) fp12q_sqr(f, qm);
    fp2 g0, g1, h1;
    miller_dbl_step_split(T, g0, g1, h1, P.x, P.y, m);
    fp12q_mul_two_lines(f, bit == 62, g0, g1, h1, qm);
    if ((X_ABS >> bit) & 1ull) {
      miller_add_step_inl(T, g0, g1, h1, Q, P.x, P.y);
      fp12q_mul_two_lines(f, false, g0, g1, h1, qm);
    }
  }
  fp12_conj(f_out, f);
  if (T_out) *T_out = T;
}
#endif

// Verify's pairing check on a lane quad: lanes 0, 1 run e(pk, H(m))'s Miller loop split, lanes 2, 3 e(-g1, sig)'s;
// the quad forms the product's halves (each pair multiplies its split value by the other pair's, the same
// product on both pairs) and both pairs run the split final exponentiation.  The signature's G2 membership comes
// from the second pair's T (g2_subgroup_from_miller).  Returns HIPBLS_OK / _ERR_SIGNATURE / _ERR_VERIFY on every
// lane of the quad.  q = lane index within the quad.
__device__ int lq4_verify(const g1a& pk, const g2a& hm, const g2a& sig, int q) {
  const uint32_t m = (q & 1) ? ~0u : 0u;
  const bool second = q >= 2;
  g1a P;
  g2a Q;
  if (second) {
    P.x = G1_GEN_X;
    P.y = G1_NEG_GEN_Y;
    Q = sig;
  } else {
    P = pk;
    Q = hm;
  }
#if BLS_LQ4_SHARED && BLS_LQ4_FE_QUAD
  const quad_m qm(q);
  fp12 r, e;
  g2j T;
  miller_loop_shared_quad(r, P, Q, qm, m, &T);
  const uint32_t mine = g2_subgroup_from_miller(T, Q) ? 1u : 0u;  // meaningful on the second pair
  const uint32_t other = quad_swap(mine);
  const uint32_t sig_in_g2 = second ? mine : other;
  final_exponentiation_quad(e, r, qm);
  const bool ok = fp12_is_one(e);
#else
  fp6 h;
  g2j T;
  miller_loop_split(h, P, Q, m, &T);
  const uint32_t mine = g2_subgroup_from_miller(T, Q) ? 1u : 0u;  // meaningful on the second pair
  const uint32_t other = quad_swap(mine);
  const uint32_t sig_in_g2 = second ? mine : other;
#endif
#if BLS_LQ4_SHARED && BLS_LQ4_FE_QUAD
#elif BLS_LQ4_FE_QUAD
  // full values: this pair's loop (gathered over the pair), the other pair's (one exchange across the pairs)
  fp12 fm, fo, f0, f1, r, e;
  fp12h_gather(fm, h, m);
  quad_swap(fo.c0, fm.c0);
  quad_swap(fo.c1, fm.c1);
  const quad_m qm(q);
  f0.c0 = sel(qm.hi, fo.c0, fm.c0);
  f0.c1 = sel(qm.hi, fo.c1, fm.c1);
  f1.c0 = sel(qm.hi, fm.c0, fo.c0);
  f1.c1 = sel(qm.hi, fm.c1, fo.c1);
  fp12q_mul(r, f0, f1, qm);
  final_exponentiation_quad(e, r, qm);
  const bool ok = fp12_is_one(e);
#else
  fp6 ho, r, e;
  for (int k = 0; k < 72; ++k) (&ho.c0.c0.v[0])[k] = quad_swap((&h.c0.c0.v[0])[k]);
  fp12h_mul(r, h, ho, m);
  final_exponentiation_split(e, r, m);
  const bool ok = fp12h_is_one(e, m);
#endif
  return !sig_in_g2 ? HIPBLS_ERR_SIGNATURE : (ok ? HIPBLS_OK : HIPBLS_ERR_VERIFY);
}

template <int MAXN>
__device__ bool lg2_check_pairs(const g1a* P, const g2a* Q, int k, uint32_t m) {
  fp12 f;
  if (k > 0)
    miller_loop_multi<MAXN>(f, P, Q, k);
  else
    fp12_set_one(f);
  return lg2_finish(f, m);
}

template <int MAXN, class GetPair>
__device__ bool pairing_check_lg2(int n, uint32_t m, GetPair get_pair) {
  const int par = m ? 1 : 0;
  g1a P[MAXN];
  g2a Q[MAXN];
  int k = 0;
  for (int i = par; i < n && k < MAXN; i += 2, ++k) get_pair(i, P[k], Q[k]);
  return lg2_check_pairs<MAXN>(P, Q, k, m);
}

// rlc_window (rlc.h) on a lane pair: both lanes form the same runs (sums of scaled keys per message run, the sum of
// scaled signatures), each converts to affine and Miller-loops only the pairs of its parity, then the split
// final exponentiation.  Same verdict as rlc_window.
template <class LoadPk, class LoadSig, class LoadH>
__device__ bool rlc_window_lg2(uint64_t i0, uint64_t i1, const int32_t* status, const uint32_t* msg_idx,
                               LoadPk load_pk, LoadSig load_sig, LoadH load_h, uint32_t m) {
  constexpr int MAXN = (RLC_W + 2) / 2;
  const int par = m ? 1 : 0;
  g1a P[MAXN];
  g2a Q[MAXN];
  int np = 0, k = 0;
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
    const uint32_t mi = msg_idx[i];
    if (mi != run_msg) {
      if (run_msg != 0xffffffffu && !jac_is_inf(run)) {
        if ((np & 1) == par) {
          jac_to_aff(P[k], run);
          load_h(Q[k], run_msg);
          ++k;
        }
        ++np;
      }
      run = qp;
      run_msg = mi;
    } else {
      jac_add(run, run, qp);
    }
  }
  if (!any) return true;
  if (!jac_is_inf(run)) {
    if ((np & 1) == par) {
      jac_to_aff(P[k], run);
      load_h(Q[k], run_msg);
      ++k;
    }
    ++np;
  }
  if (!jac_is_inf(S)) {
    if ((np & 1) == par) {
      P[k].x = G1_GEN_X;
      P[k].y = G1_NEG_GEN_Y;
      jac_to_aff(Q[k], S);
      ++k;
    }
    ++np;
  }
  if (np == 0) return true;  // np, any: same on both lanes
  return lg2_check_pairs<MAXN>(P, Q, k, m);
}

// hash_to_g2 (h2c.h) on a lane pair.  Both lanes expand the message and invert the two SSWU denominators together
// (same data, same branches); the even lane maps u0 and the odd lane u1 (SSWU + isogeny, the square-root powers
// run side by side), the pair swaps the two points after the maps have reconverged, and both lanes form
// q0 + q1 in hash_to_g2's order and clear the cofactor.  Same Jacobian result as hash_to_g2, on both lanes.
// q0 + q1 before the cofactor clearing (hash_to_g2_pair's first part; verify_lat.hip clears it on a lane quad)
BLS_CALL __device__ void hash_to_g2_pair_sum(g2j& s, const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                                             uint32_t dst_len, uint32_t m) {
  uint32_t uni[64];
  expand_message_xmd_256(uni, msg, msg_len, dst, dst_len);
  fp2 u0, u1;
  fp_from_be64_words(u0.c0, uni + 0);
  fp_from_be64_words(u0.c1, uni + 16);
  fp_from_be64_words(u1.c0, uni + 32);
  fp_from_be64_words(u1.c1, uni + 48);
  fp2 zu0, zu1, d0, d1, t0, t1, inv;
  BLS_RACE_POLL();
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
  const fp2 u = sel(m, u1, u0), zu = sel(m, zu1, zu0), t = sel(m, t1, t0);
  g2a qa;
  BLS_RACE_POLL();
  map_to_curve_sswu_tv(qa, u, zu, t);
  g2j q, qo, q0, q1;
  BLS_RACE_POLL();
  iso_map_g2(q, qa);
  pair_swap_words<72>(&qo.x.c0.v[0], &q.x.c0.v[0]);
  sel_words<72>(&q0.x.c0.v[0], m, &qo.x.c0.v[0], &q.x.c0.v[0]);  // the even lane's point (u0)
  sel_words<72>(&q1.x.c0.v[0], m, &q.x.c0.v[0], &qo.x.c0.v[0]);  // the odd lane's point (u1)
  jac_add(s, q0, q1);
}
BLS_CALL __device__ void hash_to_g2_pair(g2j& out, const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                                         uint32_t dst_len, uint32_t m) {
  g2j s;
  hash_to_g2_pair_sum(s, msg, msg_len, dst, dst_len, m);
  g2_clear_cofactor(out, s);
}

#endif  // __HIPCC__

}  // namespace bls
