// gj.h -- in-register complex Gauss-Jordan inverse + log|det| for one N x N
// matrix per wavefront (replaces jnp.linalg.slogdet, network_blocks.py:156, and
// provides B = A^{-1} for the derivative contractions).
//
// Partial pivoting is virtual (no rows move): the pivot of step k is the unused
// row with the first maximal |re|+|im| in column k (LAPACK izamax rule), the
// same rows LU partial pivoting selects.  Layout and step: see gj_inverse.
#pragma once
#include "jets.h"

namespace aq {

template <typename T> __device__ __forceinline__ T f_max(T a, T b) { return a > b ? a : b; }


// DPP row_newbcast:k (lane k of each 16-lane row to the whole row); k must fold to a
// constant (fully unrolled loops).
template <typename T> __device__ __forceinline__ T row_bcast(T x, int k) {
  switch (k) {
    case 0: return dpp<0x150>(x);
    case 1: return dpp<0x151>(x);
    case 2: return dpp<0x152>(x);
    case 3: return dpp<0x153>(x);
    case 4: return dpp<0x154>(x);
    case 5: return dpp<0x155>(x);
    case 6: return dpp<0x156>(x);
    case 7: return dpp<0x157>(x);
    case 8: return dpp<0x158>(x);
    case 9: return dpp<0x159>(x);
    case 10: return dpp<0x15A>(x);
    case 11: return dpp<0x15B>(x);
    case 12: return dpp<0x15C>(x);
    case 13: return dpp<0x15D>(x);
    case 14: return dpp<0x15E>(x);
    default: return dpp<0x15F>(x);
  }
}

// A[r][c] = Ph[r][c] * Yv[r][c]  (Ph complex interleaved [N][N][2], Yv real [N][N]).
// Writes B = A^{-1} to Bout[N][N][2]; returns log|det A| and the unit phase (phr, phi).
//
// In-place Gauss-Jordan, column layout: lane l = 16*rg + c holds column c (< N) of
// rows rg*RW .. rg*RW+RW-1 (RW = ceil(N/4)) in VGPRs.  Step k (unrolled):
//   pivot p_k = first unused row with maximal |re|+|im| in column k (izamax rule;
//     per-lane best over its rows, readlanes of the four row groups, ballot);
//   q[c]  = a[p][c] / piv (c != k),  q[k] = 1 / piv   (one ds_bpermute per component);
//   a[r][c] <- (c == k ? 0 : a[r][c]) - a[r][k] q[c] for r != p, a[p][c] <- q[c],
//     a[r][k] broadcast inside the 16-lane row by DPP row_newbcast:k.
// Only N columns are carried (the inverse builds up in the pivot columns), so no
// identity block.  With virtual pivoting X[p_k][c] = A^{-1}[k][p_c]; det A =
// sgn(p) prod_k pivot_k.
// Pivot key of a candidate: bits of |re|+|im| (monotone for non-negative floats; the
// high word for double) with the low 3 bits replaced by 4 - t, so a max over
// (row slot t, row group) picks the largest magnitude and, among equal truncated
// magnitudes, the lowest row.  0 marks used / dead rows.
__device__ __forceinline__ unsigned key_bits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ unsigned key_bits(double x) {
  return (unsigned)(__builtin_bit_cast(unsigned long long, x) >> 32);
}

// rec (optional): the pivot sequence, recorded for gj_inverse_fixed: rec[k] = row of
// step k, rec[N + k] = 1 / |pivot_k|, rec[2N] = permutation parity, rec[2N + 1] = log|det A|,
// rec[2N + 2 + k] = 1 / |pivot_k| again: the anchor a walker launch re-using this order keeps
// until partial pivoting runs again (written by lane 0).
template <typename T, int N>
__device__ __forceinline__ void gj_inverse(const T* Ph, const T* Yv, T* Bout, int lane, T& logdet, T& phr,
                                           T& phi, T* rec = nullptr) {
  constexpr int RW = (N + 3) / 4;
  const int c = lane & 15;
  const int rg = lane >> 4;
  const bool clive = c < N;
  T ar[RW], ai[RW];
  unsigned kmask[RW], kcode[RW];
  int myk[RW];
#pragma unroll
  for (int t = 0; t < RW; ++t) {
    const int r = rg * RW + t;
    const bool live = r < N;
    T a = T(0), b = T(0);
    if (live && clive) {
      const T y = Yv[r * N + c];
      a = Ph[(r * N + c) * 2] * y;
      b = Ph[(r * N + c) * 2 + 1] * y;
    }
    ar[t] = a;
    ai[t] = b;
    kmask[t] = live ? ~7u : 0u;
    kcode[t] = live ? (unsigned)(4 - t) : 0u;
    myk[t] = 0;
  }
  int myp = 0;
  unsigned used = 0;   // rows chosen so far (uniform bitmask)
  int inv = 0;         // inversions of the pivot sequence, for sgn(p)
  // log|det A| = 0.5 log prod_k |pivot_k|^2, the product carried as mantissa (in [2^-N, 1),
  // no under/overflow for N <= 16) and binary exponent: one log per matrix instead of N
  // log roundings (fp32: half the log|psi| error of summing per-pivot logs)
  T pm = T(1);
  int pe = 0;
  T pr_ = T(1), pi_ = T(0);
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // ---- pivot: first maximal |re|+|im| among the unused rows of column k
    unsigned best = 0;
#pragma unroll
    for (int t = 0; t < RW; ++t) {
      const unsigned key = (key_bits(f_abs(ar[t]) + f_abs(ai[t])) & kmask[t]) | kcode[t];
      best = best > key ? best : key;
    }
    const unsigned b0 = (unsigned)rdlane((int)best, k), b1 = (unsigned)rdlane((int)best, 16 + k);
    const unsigned b2 = (unsigned)rdlane((int)best, 32 + k), b3 = (unsigned)rdlane((int)best, 48 + k);
    const unsigned m01 = b0 > b1 ? b0 : b1, m23 = b2 > b3 ? b2 : b3;
    const unsigned m = m01 > m23 ? m01 : m23;
    const int g = b0 == m ? 0 : (b1 == m ? 1 : (b2 == m ? 2 : 3));
    const int ps = m ? 4 - (int)(m & 7u) : 0;
    const int p = g * RW + ps;
    inv += __builtin_popcount(used >> p);      // earlier pivots above p
    used |= 1u << p;
    // ---- row p of this lane's column (register ps of lane 16 g + c)
    const T sr = ar[ps], si = ai[ps];
    const T pr = rdlane(sr, 16 * g + k);
    const T pim = rdlane(si, 16 * g + k);
    const T den = pr * pr + pim * pim;
    T ir, ii, rm, lden_;
    pivot_recip(pr, pim, den, ir, ii, rm, lden_);
    if (rec && lane == 0) {
      rec[k] = T(p);
      rec[N + k] = rm;
      rec[2 * N + 2 + k] = rm;
    }
    {
      // |pivot|^2 = m 2^e formed where it cannot leave the range (pivot_mag2), branch-free:
      // carrying the frexp form out of pivot_recip's range branch instead cost 3 VGPRs and 15
      // spills in the N2 proposal instantiation, whose rare fallback inlines this function
      int e;
      pm *= pivot_mag2(pr, pim, e);
      pe += e;
    }
    {
      const T ur = pr * rm, ui = pim * rm;
      const T nr = pr_ * ur - pi_ * ui, ni = pr_ * ui + pi_ * ur;
      pr_ = nr;
      pi_ = ni;
    }
    const T q0r = __shfl(sr, 16 * g + c), q0i = __shfl(si, 16 * g + c);
    const bool ck = (c == k);
    const T qr = ck ? ir : q0r * ir - q0i * ii;
    const T qi = ck ? ii : q0r * ii + q0i * ir;
    T mqr = -qr, mqi = -qi;
    // opaque to the optimiser: keeps the updates in v_fmac form (VOP2), which can
    // take the DPP row broadcast of a[r][k] as an operand (VOP3 with neg cannot on gfx9)
    asm volatile("" : "+v"(mqr), "+v"(mqi));
    // ---- eliminate column k from every row (the pivot row is overwritten below)
#pragma unroll
    for (int t = 0; t < RW; ++t) {
      const T fr = row_bcast(ar[t], k);        // a[r][k]
      const T fi = row_bcast(ai[t], k);
      T nr = ck ? T(0) : ar[t], ni = ck ? T(0) : ai[t];
      nr = f_fma(fr, mqr, nr);                 // v_fmac with the DPP broadcast folded in
      nr = f_fma(fi, qi, nr);
      ni = f_fma(fr, mqi, ni);
      ni = f_fma(fi, mqr, ni);
      ar[t] = nr;
      ai[t] = ni;
    }
    if (rg == g) {
      ar[ps] = qr;
      ai[ps] = qi;
      myk[ps] = k;
      kmask[ps] = 0u;
      kcode[ps] = 0u;
    }
    myp = ck ? p : myp;
  }
#pragma unroll
  for (int t = 0; t < RW; ++t) {
    const int r = rg * RW + t;
    if (r < N && clive) {
      Bout[(myk[t] * N + myp) * 2] = ar[t];
      Bout[(myk[t] * N + myp) * 2 + 1] = ai[t];
    }
  }
  const T ld = T(0.5) * (f_log(pm) + T(pe) * T(0.69314718055994531));
  if (rec && lane == 0) {
    rec[2 * N] = T(inv & 1);
    rec[2 * N + 1] = ld;
  }
  if (inv & 1) {
    pr_ = -pr_;
    pi_ = -pi_;
  }
  logdet = ld;
  phr = pr_;
  phi = pi_;
}

// Gauss-Jordan with a prescribed pivot sequence (a Metropolis proposal reuses its
// walker's partial-pivoting order, recorded by gj_inverse): rows are loaded permuted,
// row slot k <- A row perm[k], so step k pivots on slot k (row group k / RW, register
// k % RW), both compile-time: no pivot search, no runtime register selection, no
// bookkeeping.  The result X = (PA)^{-1} gives B[i][perm[j]] = X[i][j]; det A =
// sgn(perm) prod pivots, accumulated relative to the walker's pivots:
// z = prod_k pivot_k / |walker pivot_k| (O(1) for a one-electron move), so
// log|det A| = log|det A_walker| + log|z| and the phase is z / |z| -- one log and one
// sqrt per matrix instead of per step.  bad = some |pivot_k| < 0.1 |walker pivot_k|, some
// |pivot_k|^2 outside the floating-point range, or z not finite (the order may not suit this
// matrix: the caller falls back to gj_inverse, which scales out-of-range pivots).
// rec: the walker's record written by gj_inverse (LDS copy).
// The elimination of gj_inverse_fixed on a matrix already in its register layout:
// a2[t] = A[rec[rg RW + t]][c] for lane 16 rg + c (zero outside the N x N block).
// rec_out (optional; a walker launch re-using its previous sweep's order): log|det A| is formed
// from this matrix's own pivots (gj_inverse's mantissa / exponent product, so that it does not
// drift from sweep to sweep through the relative form) and, unless bad, the record's magnitudes
// and log|det| are rewritten for this matrix (rec_out[N + k], rec_out[2N + 1]; the order and
// its parity are unchanged), so that the walker's proposals are relative to it.
// magoff: where the reference magnitudes 1 / |pivot_k| of the `bad` test sit in rec -- N (the
// walker's current pivots, proposals) or 2N + 2 (the anchor written when partial pivoting last
// chose the order; walker launches): measured against the anchor, a pivot cannot shrink by just
// under 10x per sweep for ever without re-pivoting (the pivots' growth stays bounded over a
// long mc_step); the phase z / |z| does not depend on the reference's scale.
template <typename T, int N>
__device__ __forceinline__ void gj_fixed_regs(typename Pair<T>::type* a2, T* Bout, int lane, const T* rec,
                                              T& logdet, T& phr, T& phi, bool& bad, T* rec_out = nullptr,
                                              int magoff = N) {
  constexpr int RW = (N + 3) / 4;
  using V2 = typename Pair<T>::type;
  const int c = lane & 15;
  const int rg = lane >> 4;
  const bool clive = c < N;
  T zr = T(1), zi = T(0);
  bool small = false;
  T pkr = T(1), pki = T(0);
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int g = k / RW, ts = k % RW;
    const T pr = rdlane(pair_re<T>(a2[ts]), 16 * g + k);
    const T pim = rdlane(pair_im<T>(a2[ts]), 16 * g + k);
    const T den = pr * pr + pim * pim;
    if (lane == k) {   // pivot k parked in lane k; the relative product is formed after the loop
      pkr = pr;
      pki = pim;
    }
    // 1 / pivot by the plain formula: a |pivot|^2 outside the float range (a far-out electron's
    // row) is caught after the loop from the parked pivots and sent to the pivoted fallback, which
    // scales it (pivot_recip_me); no range branch in this loop (it cost 3 VGPRs and 15 spills in
    // the N2 proposal instantiation)
    const T rden = f_rcp(den);
    const T ir = pr * rden, ii = -pim * rden;
    const T q0r = __shfl(pair_re<T>(a2[ts]), 16 * g + c), q0i = __shfl(pair_im<T>(a2[ts]), 16 * g + c);
    const bool ck = (c == k);
    const T qr = ck ? ir : q0r * ir - q0i * ii;
    const T qi = ck ? ii : q0r * ii + q0i * ir;
    // a[r][c] <- a[r][c] + a[r][k] m with m = -q[c] (c != k) or -q[k] - 1 (c == k: there
    // a[r][k] is the lane's own entry and the result is -a[r][k] / pivot):
    //   [re, im] += fr [mr, mi] + fi [-mi, mr]
    const T mr = ck ? -qr - T(1) : -qr, mi = -qi;
    const V2 m1 = pair_make<T>(mr, mi), m2 = pair_make<T>(-mi, mr);
#pragma unroll
    for (int t = 0; t < RW; ++t) {
      const T fr = row_bcast(pair_re<T>(a2[t]), k);
      const T fi = row_bcast(pair_im<T>(a2[t]), k);
      V2 n = pair_fma<T>(fr, m1, a2[t]);
      n = pair_fma<T>(fi, m2, n);
      a2[t] = n;
    }
    if (rg == g) a2[ts] = pair_make<T>(qr, qi);
  }
  {
    // z = prod_k pivot_k / |walker pivot_k| over lanes 0..N-1 of row 0 (row_ror tree)
    const bool pl = lane < N;
    const T sk = pl ? rec[magoff + lane] : T(0);
    T ur = pl ? pkr * sk : T(1), ui = pl ? pki * sk : T(0);
    const T dk = pkr * pkr + pki * pki;
    small = __ballot(pl && ((ur * ur + ui * ui < T(1e-2)) || !(dk >= PivRange<T>::lo && dk <= PivRange<T>::hi))) != 0;
    {
      const T xr = dpp<0x128>(ur), xi = dpp<0x128>(ui);
      const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
      ur = nr;
      ui = ni;
    }
    {
      const T xr = dpp<0x124>(ur), xi = dpp<0x124>(ui);
      const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
      ur = nr;
      ui = ni;
    }
    {
      const T xr = dpp<0x122>(ur), xi = dpp<0x122>(ui);
      const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
      ur = nr;
      ui = ni;
    }
    {
      const T xr = dpp<0x121>(ur), xi = dpp<0x121>(ui);
      const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
      ur = nr;
      ui = ni;
    }
    zr = rdlane(ur, 0);
    zi = rdlane(ui, 0);
  }
  const int pc = clive ? (int)rec[c] : 0;
#pragma unroll
  for (int t = 0; t < RW; ++t) {
    const int i = rg * RW + t;
    if (i < N && clive) {
      Bout[(i * N + pc) * 2] = pair_re<T>(a2[t]);
      Bout[(i * N + pc) * 2 + 1] = pair_im<T>(a2[t]);
    }
  }
  const T z2 = zr * zr + zi * zi;
  const bool zok = z2 > T(0) && z2 < T(1e30);
  const T rz = f_rcp(f_sqrt(zok ? z2 : T(1)));
  const T sg = rec[2 * N] != T(0) ? -rz : rz;
  logdet = rec[2 * N + 1] + T(0.5) * f_log(zok ? z2 : T(1));
  phr = zr * sg;
  phi = zi * sg;
  bad = small || !zok;
  if (rec_out) {
    const bool pl = lane < N;
    const T den = pkr * pkr + pki * pki;   // in range unless bad (then gj_inverse re-runs)
    int e = 0;
    T m = pl ? f_frexp(den, e) : T(1);
    T ef = pl ? T(e) : T(0);
    // product of the mantissas (each in [1/2, 1): no underflow for N <= 16) and sum of the
    // exponents over lanes 0..15 by the row_ror tree above
    m *= dpp<0x128>(m);
    ef += dpp<0x128>(ef);
    m *= dpp<0x124>(m);
    ef += dpp<0x124>(ef);
    m *= dpp<0x122>(m);
    ef += dpp<0x122>(ef);
    m *= dpp<0x121>(m);
    ef += dpp<0x121>(ef);
    const T ld = T(0.5) * (f_log(rdlane(m, 0)) + rdlane(ef, 0) * T(0.69314718055994531));
    logdet = ld;
    if (!bad) {
      if (pl) rec_out[N + lane] = f_sqrt(f_rcp(den));
      if (lane == 0) rec_out[2 * N + 1] = ld;
    }
  }
}

template <typename T, int N>
__device__ __forceinline__ void gj_inverse_fixed(const T* Ph, const T* Yv, T* Bout, int lane, const T* rec,
                                                 T& logdet, T& phr, T& phi, bool& bad, T* rec_out = nullptr,
                                                 int magoff = N) {
  constexpr int RW = (N + 3) / 4;
  using V2 = typename Pair<T>::type;
  const int c = lane & 15;
  const int rg = lane >> 4;
  const bool clive = c < N;
  V2 a2[RW];
#pragma unroll
  for (int t = 0; t < RW; ++t) {
    const int k = rg * RW + t;
    T a = T(0), b = T(0);
    if (k < N && clive) {
      const int r = (int)rec[k];
      const T y = Yv[r * N + c];
      a = Ph[(r * N + c) * 2] * y;
      b = Ph[(r * N + c) * 2 + 1] * y;
    }
    a2[t] = pair_make<T>(a, b);
  }
  gj_fixed_regs<T, N>(a2, Bout, lane, rec, logdet, phr, phi, bad, rec_out, magoff);
}

}  // namespace aq
