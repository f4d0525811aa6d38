// quad_small.h -- value-only log|psi| and phase of single-electron-moved configurations for
// N <= 4 electrons, FOUR configurations per wavefront (one 16-lane row each).
//
// These are the pseudopotential quadrature configurations of aiqmc_local_energy_ecp and
// aiqmc_dmc_tmoves (Energy/pphamiltonian.py:130-190, DMC/Tmoves.py:32-225): electron i of
// walker b moved to one of the N*A*50 rotated grid points.  k_walker_rev's value-only proposal
// path evaluates one configuration per 64-lane wave in the N2-sized lane layout; for the C atom
// (N = 4) that leaves 3/4 of the lanes of every phase idle (838 VALU instructions per
// configuration, 1.1 ms for the 819,200 configurations of a 4096-walker batch).  Here a 16-lane
// row holds one configuration:
//   F1 walker b's cached stage (WCache: Yt, ae features, pair column sums, J) with electron i's
//      entries from k_moved_electron's record (ECache), as the proposal path;
//   F2 the pair column sums patched with the 2(N-1) pairs of the moved electron
//      (lane 4 part + o: new/old x row/column, part 0..3);
//   F4 the three h-stream layers, lane 4i + f; the spin-group means are class sums inside the
//      16-lane row (DPP row_ror 4, 8), the conv quads as in k_walker_rev;
//   F5 Phi (x) Yt and its determinant by LU with partial pivoting (LAPACK izamax rule, virtual
//      row exchanges) inside one quad: lane c of the row's first quad holds column c, column k
//      is broadcast by DPP quad_perm.  No inverse is needed for values, so no fixed pivot order
//      and no fallback.
// log|psi| = log|det| + J_ae + J_ee (the Jastrows multiply the matrix, nn.py:504, Q11).
#pragma once
#include "walker_rev.h"

namespace aq {

// sum over the 16 lanes of this lane's row (every lane receives the total)
template <typename T> __device__ __forceinline__ T row16_sum(T x) {
  x += dpp<0x128>(x);
  x += dpp<0x124>(x);
  x += dpp<0x122>(x);
  x += dpp<0x121>(x);
  return x;
}
// sum over the lanes 4i + f of this lane's row with equal f (over electrons i, per unit f)
template <typename T> __device__ __forceinline__ T row_class4_sum(T x) {
  x += dpp<0x124>(x);
  x += dpp<0x128>(x);
  return x;
}

// per-row (configuration) LDS block
template <typename T, int N, int A>
struct SmemQ {
  static constexpr int D0 = 4 * A;
  static constexpr int xs = 0;                    // [3N]      positions, the moved electron at its new place
  static constexpr int xo = xs + 12;              // [3]       old position of the moved electron
  static constexpr int yv = xo + 4;               // [N][N]    Yt
  static constexpr int hl = yv + 16;              // [N][D0]   ae features
  static constexpr int g2 = hl + 4 * D0;          // [3][2][N][4] pair column means
  static constexpr int S = g2 + 3 * 2 * 4 * 4;    // [16][12]  pair values of the patch
  static constexpr int h3 = S + 16 * 12;          // [N][4]    h-stream output
  static constexpr int size = h3 + 16;
};

// waves per workgroup (independent; the launch pays per workgroup, see walker_rev.h AQ_PROP_WPB)
constexpr int QUAD_WPB = 1;   // 4 measured 0.354 vs 0.346 ms (C atom): per-workgroup cost is not the limit here

template <typename T, int N, int A>
__global__ __launch_bounds__(64 * QUAD_WPB) void k_quad_value(KArgs ka) {
  static_assert(N <= 4, "four configurations per wave need N <= 4");
  using Ly = Lay<N, A>;
  using WC = WCache<N, A>;
  using EC = ECache<N, A>;
  using SQ = SmemQ<T, N, A>;
  constexpr int D0 = 4 * A;
  const cptr<T> P = param_ptr<T>(ka.prm);
  __shared__ T smq[QUAD_WPB * 4 * SQ::size];
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int slot = lane >> 4, sl = lane & 15;
  const int c0 = (xcd_major(blockIdx.x, gridDim.x) * QUAD_WPB + wv) * 4 + slot;
  const bool act = c0 < ka.nconf;
  const int conf = act ? c0 : ka.nconf - 1;
  T* sm = smq + (wv * 4 + slot) * SQ::size;
  T* xs = sm + SQ::xs;
  T* Yv = sm + SQ::yv;
  T* hl = sm + SQ::hl;
  T* g2 = sm + SQ::g2;
  T* S = sm + SQ::S;
  T* H3 = sm + SQ::h3;
  const int mper = ka.mper ? ka.mper : N, mdiv = ka.mdiv ? ka.mdiv : 1;
  const int pb = conf / mper, pi = (conf - pb * mper) / mdiv;
  const int nup = ka.nup;
  const T RSQ2 = T(0.70710678118654752);
  const T ginv0 = T(1) / T(nup), ginv1 = T(1) / T(N - nup);
  const T* Wc = (const T*)ka.wcache + (size_t)pb * WC::size;
  const T* Eq = (const T*)ka.ecache + (size_t)conf * EC::size;

  // ---------------------------------------------------------------- F1 cached stage of walker pb
  if (sl < 3 * N) {
    const T x0 = ((const T*)ka.pos)[(size_t)pb * 3 * N + sl];
    const bool mv = sl / 3 == pi;
    if (mv) sm[SQ::xo + sl - 3 * pi] = x0;
    xs[sl] = mv ? Eq[EC::xp + sl - 3 * pi] : x0;
  }
  if (sl < N * N) {
    const int r = sl / N;
    Yv[sl] = r == pi ? Eq[EC::yv + sl - r * N] : Wc[WC::yv + sl];
  }
  for (int idx = sl; idx < N * D0; idx += 16) {
    const int e = idx / D0;
    hl[idx] = e == pi ? Eq[EC::h0 + idx - e * D0] : Wc[WC::h0 + idx];
  }
  for (int idx = sl; idx < 3 * 2 * N * 4; idx += 16) g2[idx] = Wc[WC::g2 + idx];
  T jsum = sl < N ? (sl == pi ? Eq[EC::jv] : Wc[WC::jaev + sl]) : T(0);
  if (sl == 0) jsum += Wc[WC::jee];
  wave_sync();

  // ---------------------------------------------------------------- F2 pairs of the moved electron
  // lane 4 part + o: part 0/1 pair (pi, o) at the new/old x_pi (column o), part 2/3 pair (o, pi)
  {
    const int part = sl >> 2, o = sl & 3;
    const int os = o < N ? o : N - 1;
    const T* xp = (part & 1) ? sm + SQ::xo : xs + pi * 3;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = part < 2 ? xs[os * 3 + c] - xp[c] : xp[c] - xs[os * 3 + c];
    T v[3][4];
    pair_values<T, N, A>(d, P, v);
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int f = 0; f < 4; ++f) S[sl * 12 + l * 4 + f] = v[l][f];
    if (part < 2 && o < N && o != pi) {
      const T cusp = P[Ly::jee_c + pi * N + o], al = P[Ly::jee_a + pi * N + o];
      const T je = f_div(cusp * v[0][0], al * v[0][0] + T(1));
      jsum += part == 0 ? je : -je;
    }
  }
  wave_sync();
  if (sl < N && sl != pi) {
    const int Gp = pi >= nup ? 1 : 0;
    const T gw = Gp ? ginv1 : ginv0;
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        g2[((l * 2 + Gp) * N + sl) * 4 + f] += (S[sl * 12 + l * 4 + f] - S[(4 + sl) * 12 + l * 4 + f]) * gw;
  }
#pragma unroll
  for (int t0 = 0; t0 < 24; t0 += 16) {
    const int t = t0 + sl;
    if (t < 24) {
      const int l = t >> 3, G = (t >> 2) & 1, f = t & 3;
      const int k0 = G ? nup : 0, k1 = G ? N : nup;
      T acc = T(0);
      for (int k = k0; k < k1; ++k)
        if (k != pi) acc += S[(8 + k) * 12 + l * 4 + f] - S[(12 + k) * 12 + l * 4 + f];
      g2[((l * 2 + G) * N + pi) * 4 + f] += acc * (G ? ginv1 : ginv0);
    }
  }
  wave_sync();

  // ---------------------------------------------------------------- F4 h-stream layers
  // (the arithmetic of k_walker_rev's F4, lane 4i + f inside the row)
  const int fi = sl >> 2, ff = sl & 3;
  const bool ilive = fi < N;
  const int ic = ilive ? fi : N - 1;
  const bool inG1 = ic >= nup;
  constexpr int QM = (3 * D0 + 8) / 4;
  T hreg = T(0);
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const int d1 = l == 0 ? D0 : NH;
    const int DF = 3 * d1 + 8;
    const int Q = DF / 4;
    const int T4 = d1 / 4;
    const cptr<T> convw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2)) + ic * DF;
    const cptr<T> convb = P + (l == 0 ? Ly::conv_b0 : (l == 1 ? Ly::conv_b1 : Ly::conv_b2)) + ic * Q;
    const cptr<T> sngw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
    const cptr<T> sngb = P + (l == 0 ? Ly::sng_b0 : (l == 1 ? Ly::sng_b1 : Ly::sng_b2));
    T hown[D0 / 4];
#pragma unroll
    for (int t = 0; t < D0 / 4; ++t) hown[t] = l == 0 ? hl[ic * D0 + ff + 4 * t] : hreg;
    T gown[2][D0 / 4];
#pragma unroll
    for (int t = 0; t < D0 / 4; ++t) {
      if (t < T4) {
        const T x = ilive ? hown[t] : T(0);
        gown[0][t] = row_class4_sum(inG1 ? T(0) : x) * ginv0;
        gown[1][t] = row_class4_sum(inG1 ? x : T(0)) * ginv1;
      }
    }
    T zc[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q < Q) {
        T F;
        if (q < T4) F = hown[q];
        else if (q < 3 * T4) F = gown[(q - T4) / T4][(q - T4) % T4];
        else F = g2[((l * 2 + (q - 3 * T4)) * N + ic) * 4 + ff];
        T z = F * convw[4 * q + ff];
        z += dpp<0xB1>(z);
        z += dpp<0x4E>(z);
        zc[q] = z;
      }
    }
    const int QF = Q / 4;
    T cq[QM];
#pragma unroll
    for (int s4 = 0; s4 < QM / 4; ++s4) {
      if (s4 < QF) {
        const int q0 = 4 * s4;
        const T zs = ff == 0 ? zc[q0] : (ff == 1 ? zc[q0 + 1] : (ff == 2 ? zc[q0 + 2] : zc[q0 + 3]));
        const T c = f_tanh(zs * T(0.25) + convb[q0 + ff]);
        cq[q0 + 0] = quad_bcast<0>(c);
        cq[q0 + 1] = quad_bcast<1>(c);
        cq[q0 + 2] = quad_bcast<2>(c);
        cq[q0 + 3] = quad_bcast<3>(c);
      }
    }
#pragma unroll
    for (int q = 0; q < QM; ++q)
      if (q >= 4 * QF && q < Q) cq[q] = f_tanh(zc[q] * T(0.25) + convb[q]);
    T z = sngb[ff], z1 = T(0);
#pragma unroll
    for (int q = 0; q < QM; ++q)
      if (q < Q) {
        if (q & 1) z1 += cq[q] * sngw[q * 4 + ff];
        else z += cq[q] * sngw[q * 4 + ff];
      }
    z += z1;
    const T sval = f_tanh(z);
    const T hin = l == 0 ? hl[ic * D0 + ff] : hreg;
    hreg = (d1 == NH) ? (hin + sval) * RSQ2 : sval;
  }
  if (ilive) H3[ic * 4 + ff] = hreg;
  wave_sync();

  // ---------------------------------------------------------------- F5 log det(Phi (x) Yt), LU in a quad
  T lsum = T(0), ur = T(1), ui = T(0);
  int inv = 0;
  if (sl < 4) {
    const int c = sl;
    const int* rowsrc = ka.rowsrc;
    T ar[4], ai[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      T a = T(0), b = T(0);
      if (r < N && c < N) {
        const int src = rowsrc[r];
        const int sp = r < nup ? 0 : 1;
        T re = P[Ly::orb_b + (sp * N + c) * 2 + 0], im = P[Ly::orb_b + (sp * N + c) * 2 + 1];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const T hv = H3[src * 4 + f];
          re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 0];
          im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1];
        }
        const T y = Yv[r * N + c];
        a = re * y;
        b = im * y;
      }
      ar[r] = a;
      ai[r] = b;
    }
    unsigned used = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      // column k of every row, from lane k of the quad
      T kr[4], ki[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kr[r] = k == 0 ? quad_bcast<0>(ar[r]) : (k == 1 ? quad_bcast<1>(ar[r]) : (k == 2 ? quad_bcast<2>(ar[r]) : quad_bcast<3>(ar[r])));
        ki[r] = k == 0 ? quad_bcast<0>(ai[r]) : (k == 1 ? quad_bcast<1>(ai[r]) : (k == 2 ? quad_bcast<2>(ai[r]) : quad_bcast<3>(ai[r])));
      }
      // pivot: first unused row with the largest |re| + |im| (izamax)
      int p = 0;
      T best = T(-1);
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const T m = f_abs(kr[r]) + f_abs(ki[r]);
        const bool take = !((used >> r) & 1u) && m > best;
        best = take ? m : best;
        p = take ? r : p;
      }
      T pr = T(0), pim = T(0), rpr = T(0), rpi = T(0);   // pivot, this lane's entry of row p
#pragma unroll
      for (int r = 0; r < N; ++r)
        if (r == p) {
          pr = kr[r];
          pim = ki[r];
          rpr = ar[r];
          rpi = ai[r];
        }
      inv += __builtin_popcount(used >> p);   // earlier pivots below p in the row order
      used |= 1u << p;
      const T den = pr * pr + pim * pim;
      const T rden = f_rcp(den);
      lsum += f_log(den);
      {
        const T rm = f_sqrt(rden);
        const T xr = pr * rm, xi = pim * rm;
        const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
        ur = nr;
        ui = ni;
      }
      const T ipr = pr * rden, ipi = -pim * rden;   // 1 / pivot
#pragma unroll
      for (int r = 0; r < N; ++r) {
        if (!((used >> r) & 1u)) {
          const T mr = kr[r] * ipr - ki[r] * ipi, mi = kr[r] * ipi + ki[r] * ipr;
          ar[r] -= mr * rpr - mi * rpi;
          ai[r] -= mr * rpi + mi * rpr;
        }
      }
    }
  }
  const T jt = row16_sum(jsum);
  if (act && sl == 0) {
    const T sg = (inv & 1) ? T(-1) : T(1);
    if (ka.logabs) ((T*)ka.logabs)[conf] = T(0.5) * lsum + jt;
    if (ka.phase) ((T*)ka.phase)[conf] = f_atan2(ui * sg, ur * sg);
  }
}

}  // namespace aq
