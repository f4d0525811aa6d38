// quad_small.h -- single-electron-moved configurations and walkers of small systems, several
// configurations per wavefront.
//
// k_quad_value: value-only log|psi| and phase of the pseudopotential quadrature configurations of
// aiqmc_local_energy_ecp and aiqmc_dmc_tmoves (Energy/pphamiltonian.py:130-190,
// DMC/Tmoves.py:32-225): electron i of walker b moved to one of the N*A*50 rotated grid points.
// k_walker_rev's value-only proposal path evaluates one configuration per 64-lane wave in the
// N2-sized lane layout; for the C atom (N = 4) that leaves 3/4 of the lanes of every phase idle
// (838 VALU instructions per configuration, 1.1 ms for the 819,200 configurations of a
// 4096-walker batch).  Here a slot of SW lanes holds one configuration (SW = 16 for N <= 4: four
// per wave; SW = 32 for N <= 8: two per wave):
//   F1 walker b's cached stage (WCache: Yt, ae features, pair column sums, J) with electron i's
//      entries from the moved-electron record (ECache), as the proposal path;
//   F2 the pair column sums patched with the 2(N-1) pairs of the moved electron
//      (lane NI part + o: new/old x row/column, part 0..3);
//   F4 the three h-stream layers, lane 4i + f; the spin-group means are class sums inside the
//      slot (DPP row_ror 4, 8, and a lane swizzle across the two rows of a 32-lane slot), the
//      conv quads as in k_walker_rev;
//   F5 Phi (x) Yt and its determinant by LU with partial pivoting (LAPACK izamax rule, virtual
//      row exchanges): lane 4r + c of the slot holds row r's entries c (and c + 4 for N > 4),
//      column k reaches row r's lanes by quad broadcast, the pivot by a packed-key max over the
//      row quads.  No inverse is needed for values, so no fixed pivot order and no fallback.
// k_quad_grad (N <= 4, four per wave): the Metropolis proposals (value + gradient) and, WALK,
// the walker launches -- see its own header below.
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

// configurations per wave: 4 (one 16-lane row each) for N <= 4, 2 (one 32-lane half each) for
// N <= 8; NI = SW / 4 electron slots per configuration
template <int N> struct QSlot {
  static constexpr int SW = N <= 4 ? 16 : 32;
  static constexpr int NI = SW / 4;
  static constexpr int NSL = 64 / SW;
};
// sum over the SW lanes of this configuration's slot
template <int SW, typename T> __device__ __forceinline__ T slot_sum(T x) {
  x = row16_sum(x);
  if constexpr (SW == 32) x += __shfl_xor(x, 16);
  return x;
}
// sum over the slot's lanes 4i + f with equal f (over electrons i, per unit f)
template <int SW, typename T> __device__ __forceinline__ T slot_class4_sum(T x) {
  x = row_class4_sum(x);
  if constexpr (SW == 32) x += __shfl_xor(x, 16);
  return x;
}

// per-slot (configuration) LDS block
template <typename T, int N, int A>
struct SmemQ {
  static constexpr int D0 = 4 * A;
  static constexpr int NI = QSlot<N>::NI, SW = QSlot<N>::SW;
  static constexpr int xs = 0;                    // [3N]      positions, the moved electron at its new place
  static constexpr int xo = xs + 3 * NI;          // [3]       old position of the moved electron
  static constexpr int yv = xo + 4;               // [N][N]    Yt
  static constexpr int hl = yv + NI * NI;         // [N][D0]   ae features
  static constexpr int g2 = hl + NI * D0;         // [3][2][N][4] pair column means
  static constexpr int S = g2 + 3 * 2 * NI * 4;   // [NI][12]  new - old pair values (o, pi) of the patch
  static constexpr int h3 = S + NI * 12;          // [N][4]    h-stream output
  static constexpr int pv = h3 + NI * 4;          // [2N+1]    the walker's pivot record (fixed-order LU)
  static constexpr int size = pv + 2 * NI + 4;
};

// k_quad_value's determinant by LU in the walker's pivot order (the record its walker launch wrote,
// gj.h layout: row of step k, 1 / |pivot_k|, the order's parity) instead of partial pivoting: no
// pivot search per step.  A slot whose pivot k falls below 0.1 of its walker's (or out of the float
// range) reruns the pivoted LU.  A quadrature configuration moves one electron far (onto the sphere
// around an atom), and still 2.9 % of C2 ccECP configurations need the rerun (CPU experiment on the
// fp64 oracle's matrices).  -DAQ_QUAD_PIVOTED: the pivoted LU always.
#ifndef AQ_QUAD_PIVOTED
constexpr bool kQuadFixedLU = true;
#else
constexpr bool kQuadFixedLU = false;
#endif

// F1 of the packed kernels: walker pb's cached stage (positions X, walker cache Wc) with electron
// pi's entries from its moved-electron record Eq, into the slot's LDS block.  Every load is
// issued (at clamped in-bounds addresses; the moved electron's entries by one load from a
// selected address) before the first LDS write, so a slot pays one memory round trip instead of
// one per loop trip.  Returns this lane's share of J (J_ae of electron sl, + J_ee on lane 0).
template <typename T, int N, int A, int SW>
__device__ __forceinline__ T quad_stage_load(const T* X, const T* Wc, const T* Eq, int pi, int sl, T* xs, T* xo,
                                             T* Yv, T* hl, T* g2) {
  using WC = WCache<N, A>;
  using EC = ECache<N, A>;
  constexpr int D0 = 4 * A;
  constexpr int NX = (3 * N + SW - 1) / SW, NY = (N * N + SW - 1) / SW, NHL = (N * D0 + SW - 1) / SW;
  constexpr int NG = (24 * N + SW - 1) / SW;
  T x0[NX], xv[NX], yv[NY], hv[NHL], gv[NG];
#pragma unroll
  for (int t = 0; t < NX; ++t) {
    const int idx = sl + t * SW, ic = idx < 3 * N ? idx : 3 * N - 1;
    x0[t] = X[ic];
    xv[t] = *(ic / 3 == pi ? Eq + EC::xp + ic % 3 : X + ic);
  }
#pragma unroll
  for (int t = 0; t < NY; ++t) {
    const int idx = sl + t * SW, ic = idx < N * N ? idx : N * N - 1;
    yv[t] = *(ic / N == pi ? Eq + EC::yv + ic % N : Wc + WC::yv + ic);
  }
#pragma unroll
  for (int t = 0; t < NHL; ++t) {
    const int idx = sl + t * SW, ic = idx < N * D0 ? idx : N * D0 - 1;
    hv[t] = *(ic / D0 == pi ? Eq + EC::h0 + ic % D0 : Wc + WC::h0 + ic);
  }
#pragma unroll
  for (int t = 0; t < NG; ++t) {
    const int idx = sl + t * SW;
    gv[t] = Wc[WC::g2 + (idx < 24 * N ? idx : 24 * N - 1)];
  }
  const int jc = sl < N ? sl : N - 1;
  const T jv = *(jc == pi ? Eq + EC::jv : Wc + WC::jaev + jc);
  const T jee = Wc[WC::jee];
#pragma unroll
  for (int t = 0; t < NX; ++t) {
    const int idx = sl + t * SW;
    if (idx < 3 * N) {
      if (idx / 3 == pi) xo[idx - 3 * pi] = x0[t];
      xs[idx] = xv[t];
    }
  }
#pragma unroll
  for (int t = 0; t < NY; ++t)
    if (sl + t * SW < N * N) Yv[sl + t * SW] = yv[t];
#pragma unroll
  for (int t = 0; t < NHL; ++t)
    if (sl + t * SW < N * D0) hl[sl + t * SW] = hv[t];
#pragma unroll
  for (int t = 0; t < NG; ++t)
    if (sl + t * SW < 24 * N) g2[sl + t * SW] = gv[t];
  T jsum = sl < N ? jv : T(0);
  if (sl == 0) jsum += jee;
  return jsum;
}

template <typename T, int N, int A>
__global__ __launch_bounds__(64) void k_quad_value(KArgs ka) {
  static_assert(N <= 8, "several configurations per wave need N <= 8");
  using Ly = Lay<N, A>;
  using WC = WCache<N, A>;
  using EC = ECache<N, A>;
  using SQ = SmemQ<T, N, A>;
  constexpr int D0 = 4 * A;
  constexpr int SW = QSlot<N>::SW, NI = QSlot<N>::NI, NSL = QSlot<N>::NSL;
  const cptr<T> P = param_ptr<T>(ka.prm);
  __shared__ T smq[NSL * SQ::size];
  const int lane = threadIdx.x;
  const int slot = lane / SW, sl = lane % SW;
  const int c0 = xcd_major(blockIdx.x, gridDim.x) * NSL + slot;
  const bool act = c0 < ka.nconf;
  const int conf = act ? c0 : ka.nconf - 1;
  T* sm = smq + slot * SQ::size;
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
  T jsum = quad_stage_load<T, N, A, SW>((const T*)ka.pos + (size_t)pb * 3 * N, Wc, Eq, pi, sl, xs, sm + SQ::xo,
                                        Yv, hl, g2);
  if constexpr (kQuadFixedLU) {   // the walker's pivot record (order, 1 / |pivot|, parity) for F5
    const T v = Wc[WC::pv + (sl < 2 * N + 1 ? sl : 2 * N)];
    if (sl < 2 * N + 1) sm[SQ::pv + sl] = v;
  }
  wave_sync();

  // ---------------------------------------------------------------- F2 pairs of the moved electron
  // lane NI part + o: part 0/1 pair (pi, o) at the new/old x_pi (column o), part 2/3 pair (o, pi);
  // new - old by one DPP row shift (lane + NI, inside the lane's 16-lane row), part 0 into the
  // pair column means of row o, part 2 into S for the row-pi sums
  {
    const int part = sl / NI, o = sl % NI;
    const int os = o < N ? o : N - 1;
    const T* xp = (part & 1) ? sm + SQ::xo : xs + pi * 3;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = part < 2 ? xs[os * 3 + c] - xp[c] : xp[c] - xs[os * 3 + c];
    T v[3][4];
    pair_values<T, N, A>(d, P, v);
    T dv[3][4];
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int f = 0; f < 4; ++f) dv[l][f] = v[l][f] - dpp<0x100 + NI>(v[l][f]);
    if (part < 2 && o < N && o != pi) {
      const T cusp = P[Ly::jee_c + pi * N + o], al = P[Ly::jee_a + pi * N + o];
      const T je = f_div(cusp * v[0][0], al * v[0][0] + T(1));
      jsum += part == 0 ? je : -je;
    }
    if (part == 0 && o < N && o != pi) {
      const int Gp = pi >= nup ? 1 : 0;
      const T gw = Gp ? ginv1 : ginv0;
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int f = 0; f < 4; ++f) g2[((l * 2 + Gp) * N + o) * 4 + f] += dv[l][f] * gw;
    }
    if (part == 2) {
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int f = 0; f < 4; ++f) S[o * 12 + l * 4 + f] = dv[l][f];
    }
  }
  wave_sync();
#pragma unroll
  for (int t0 = 0; t0 < 24; t0 += SW) {
    const int t = t0 + sl;
    if (t < 24) {
      const int l = t >> 3, G = (t >> 2) & 1, f = t & 3;
      const int k0 = G ? nup : 0, k1 = G ? N : nup;
      T acc = T(0);
      for (int k = k0; k < k1; ++k)
        if (k != pi) acc += S[k * 12 + l * 4 + f];
      g2[((l * 2 + G) * N + pi) * 4 + f] += acc * (G ? ginv1 : ginv0);
    }
  }
  wave_sync();

  // ---------------------------------------------------------------- F4 h-stream layers
  // (the arithmetic of k_walker_rev's F4, lane 4i + f inside the slot)
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
        gown[0][t] = slot_class4_sum<SW>(inG1 ? T(0) : x) * ginv0;
        gown[1][t] = slot_class4_sum<SW>(inG1 ? x : T(0)) * ginv1;
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

  // ---------------------------------------------------------------- F5 log det(Phi (x) Yt), LU in a row
  // lane c < NI of the slot's first 16-lane row holds column c; column k comes by DPP row_newbcast
  T lsum = T(0), ur = T(1), ui = T(0);
  int inv = 0;
  // one LU step's pivot bookkeeping: log|pivot|^2, the running phase, 1 / pivot
  auto pivot_step = [&](T pr, T pim, T& ipr, T& ipi, T& rabs) {
    const T den = pr * pr + pim * pim;
    T lden;
    pivot_recip(pr, pim, den, ipr, ipi, rabs, lden);
    lsum += lden;
    const T xr = pr * rabs, xi = pim * rabs;
    const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
    ur = nr;
    ui = ni;
  };
  if constexpr (SW == 16) {
    // N <= 4: one element per lane, lane 4r + c of the row holds A[r][c].  The pivot row of
    // column k is the max of packed keys over the column's four lanes (bits of |re| + |im| with
    // the low two bits replaced by 3 - r: the first maximal row, the izamax rule up to the two
    // dropped mantissa bits, as gj.h), two DPP row rotations; the pivot comes by row_newbcast,
    // the pivot row's entry of this lane's column by one lane permute.
    const int r = sl >> 2, c = sl & 3;
    const bool rl = r < N;
    T a0 = T(0), b0 = T(0);
    if (rl && c < N) {
      const int src = ka.rowsrc[r];
      const int sp = r < nup ? 0 : 1;
      T re = P[Ly::orb_b + (sp * N + c) * 2 + 0], im = P[Ly::orb_b + (sp * N + c) * 2 + 1];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const T hv = H3[src * 4 + f];
        re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 0];
        im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1];
      }
      const T y = Yv[r * N + c];
      a0 = re * y;
      b0 = im * y;
    }
    const int rowbase = lane & ~15;
    auto pivoted = [&]() {
      T a = a0, b = b0;
      lsum = T(0);
      ur = T(1);
      ui = T(0);
      inv = 0;
      unsigned used = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const T akr = k == 0 ? quad_bcast<0>(a) : (k == 1 ? quad_bcast<1>(a) : (k == 2 ? quad_bcast<2>(a) : quad_bcast<3>(a)));
        const T aki = k == 0 ? quad_bcast<0>(b) : (k == 1 ? quad_bcast<1>(b) : (k == 2 ? quad_bcast<2>(b) : quad_bcast<3>(b)));
        const bool open = rl && !((used >> r) & 1u);
        unsigned key = open ? ((key_bits(f_abs(akr) + f_abs(aki)) & ~3u) | (unsigned)(3 - r)) : 0u;
        {
          const unsigned k4 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x124, 0xF, 0xF, true);
          key = key > k4 ? key : k4;
          const unsigned k8 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x128, 0xF, 0xF, true);
          key = key > k8 ? key : k8;
        }
        const int p = 3 - (int)(key & 3u);
        const T p0r = row_bcast(a, k), p1r = row_bcast(a, 4 + k), p2r = row_bcast(a, 8 + k), p3r = row_bcast(a, 12 + k);
        const T p0i = row_bcast(b, k), p1i = row_bcast(b, 4 + k), p2i = row_bcast(b, 8 + k), p3i = row_bcast(b, 12 + k);
        const T pr = p == 0 ? p0r : (p == 1 ? p1r : (p == 2 ? p2r : p3r));
        const T pim = p == 0 ? p0i : (p == 1 ? p1i : (p == 2 ? p2i : p3i));
        const T er = __shfl(a, rowbase + 4 * p + c), ei = __shfl(b, rowbase + 4 * p + c);   // A[p][c]
        inv += __builtin_popcount(used >> p);
        used |= 1u << p;
        T ipr, ipi, rabs;
        pivot_step(pr, pim, ipr, ipi, rabs);   // 1 / pivot
        if (rl && !((used >> r) & 1u)) {   // rows still open: A[r][:] -= (A[r][k] / pivot) A[p][:]
          const T mr = akr * ipr - aki * ipi, mi = akr * ipi + aki * ipr;
          a -= mr * er - mi * ei;
          b -= mr * ei + mi * er;
        }
      }
    };
    if constexpr (kQuadFixedLU) {
      // the walker's order: pivot row p of step k and 1 / |walker pivot k| from the slot's LDS copy
      T a = a0, b = b0;
      bool bad = ka.quad_pivoted != 0, done = false;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const T akr = k == 0 ? quad_bcast<0>(a) : (k == 1 ? quad_bcast<1>(a) : (k == 2 ? quad_bcast<2>(a) : quad_bcast<3>(a)));
        const T aki = k == 0 ? quad_bcast<0>(b) : (k == 1 ? quad_bcast<1>(b) : (k == 2 ? quad_bcast<2>(b) : quad_bcast<3>(b)));
        const int p = (int)sm[SQ::pv + k];
        const T rk = sm[SQ::pv + N + k];
        const T er = __shfl(a, rowbase + 4 * p + c), ei = __shfl(b, rowbase + 4 * p + c);   // A[p][c]
        // A[p][k]: lane c = k of this quad holds it in er
        const T pr = k == 0 ? quad_bcast<0>(er) : (k == 1 ? quad_bcast<1>(er) : (k == 2 ? quad_bcast<2>(er) : quad_bcast<3>(er)));
        const T pim = k == 0 ? quad_bcast<0>(ei) : (k == 1 ? quad_bcast<1>(ei) : (k == 2 ? quad_bcast<2>(ei) : quad_bcast<3>(ei)));
        done = done || (p == r);
        T ipr, ipi, rabs;
        pivot_step(pr, pim, ipr, ipi, rabs);
        bad = bad || !(rk >= T(0.1) * rabs);   // |pivot| below 0.1 of the walker's (or not finite)
        if (rl && !done) {
          const T mr = akr * ipr - aki * ipi, mi = akr * ipi + aki * ipr;
          a -= mr * er - mi * ei;
          b -= mr * ei + mi * er;
        }
      }
      inv = (int)sm[SQ::pv + 2 * N];
      const unsigned long long bm = __ballot(bad);
      if ((bm >> (lane & ~(SW - 1))) & ((1ull << SW) - 1ull)) pivoted();   // this slot: partial pivoting
    } else {
      pivoted();
    }
  } else {
    // 5 <= N <= 8: lane 4r + g of the slot holds A[r][g] and A[r][g + 4] (row r, two columns).
    // Column k reaches the lanes of its row by one quad broadcast; the pivot of column k is the
    // max of packed keys (low three bits 7 - r) over the slot's eight row quads: DPP row_ror 4,
    // 8 inside each 16-lane row, one lane exchange across the slot's two rows; the pivot row's
    // two entries of this lane's columns come by lane permutes.
    const int r = sl >> 2, g = sl & 3;
    const bool rl = r < N;
    T a0[2], b0[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = g + 4 * h;
      a0[h] = T(0);
      b0[h] = T(0);
      if (rl && c < N) {
        const int src = ka.rowsrc[r];
        const int sp = r < nup ? 0 : 1;
        T re = P[Ly::orb_b + (sp * N + c) * 2 + 0], im = P[Ly::orb_b + (sp * N + c) * 2 + 1];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const T hv = H3[src * 4 + f];
          re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 0];
          im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1];
        }
        const T y = Yv[r * N + c];
        a0[h] = re * y;
        b0[h] = im * y;
      }
    }
    const int sbase = lane & ~31;
    // one step of either order: eliminate column k with pivot row p (rows still open: A[r][:] -=
    // (A[r][k] / pivot) A[p][:])
    auto lu_step = [&](int k, int p, T* a, T* b, bool open_after, T akr, T aki, T& rabs) {
      const int kh = k >> 2;
      const int srcl = sbase + 4 * p + g;
      const T er0 = __shfl(a[0], srcl), ei0 = __shfl(b[0], srcl);   // A[p][g]
      const T er1 = __shfl(a[1], srcl), ei1 = __shfl(b[1], srcl);   // A[p][g + 4]
      T pr, pim;   // A[p][k]
      {
        const T sr = kh ? er1 : er0, si = kh ? ei1 : ei0;
        if ((k & 3) == 0) { pr = quad_bcast<0>(sr); pim = quad_bcast<0>(si); }
        else if ((k & 3) == 1) { pr = quad_bcast<1>(sr); pim = quad_bcast<1>(si); }
        else if ((k & 3) == 2) { pr = quad_bcast<2>(sr); pim = quad_bcast<2>(si); }
        else { pr = quad_bcast<3>(sr); pim = quad_bcast<3>(si); }
      }
      T ipr, ipi;
      pivot_step(pr, pim, ipr, ipi, rabs);   // 1 / pivot
      if (open_after) {
        const T mr = akr * ipr - aki * ipi, mi = akr * ipi + aki * ipr;
        a[0] -= mr * er0 - mi * ei0;
        b[0] -= mr * ei0 + mi * er0;
        a[1] -= mr * er1 - mi * ei1;
        b[1] -= mr * ei1 + mi * er1;
      }
    };
    auto col_k = [&](int k, const T* a, const T* b, T& akr, T& aki) {   // A[r][k]
      const int kh = k >> 2;
      if ((k & 3) == 0) { akr = quad_bcast<0>(a[kh]); aki = quad_bcast<0>(b[kh]); }
      else if ((k & 3) == 1) { akr = quad_bcast<1>(a[kh]); aki = quad_bcast<1>(b[kh]); }
      else if ((k & 3) == 2) { akr = quad_bcast<2>(a[kh]); aki = quad_bcast<2>(b[kh]); }
      else { akr = quad_bcast<3>(a[kh]); aki = quad_bcast<3>(b[kh]); }
    };
    auto pivoted = [&]() {
      T a[2] = {a0[0], a0[1]}, b[2] = {b0[0], b0[1]};
      lsum = T(0);
      ur = T(1);
      ui = T(0);
      inv = 0;
      unsigned used = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        T akr, aki;
        col_k(k, a, b, akr, aki);
        const bool open = rl && !((used >> r) & 1u);
        unsigned key = open ? ((key_bits(f_abs(akr) + f_abs(aki)) & ~7u) | (unsigned)(7 - r)) : 0u;
        {
          const unsigned k4 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x124, 0xF, 0xF, true);
          key = key > k4 ? key : k4;
          const unsigned k8 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x128, 0xF, 0xF, true);
          key = key > k8 ? key : k8;
          const unsigned k16 = (unsigned)__shfl_xor((int)key, 16);
          key = key > k16 ? key : k16;
        }
        const int p = 7 - (int)(key & 7u);
        inv += __builtin_popcount(used >> p);   // earlier pivots below p in the row order
        used |= 1u << p;
        T rabs;
        lu_step(k, p, a, b, rl && !((used >> r) & 1u), akr, aki, rabs);
      }
    };
    if constexpr (kQuadFixedLU) {
      T a[2] = {a0[0], a0[1]}, b[2] = {b0[0], b0[1]};
      bool bad = ka.quad_pivoted != 0, done = false;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        T akr, aki;
        col_k(k, a, b, akr, aki);
        const int p = (int)sm[SQ::pv + k];
        const T rk = sm[SQ::pv + N + k];
        done = done || (p == r);
        T rabs;
        lu_step(k, p, a, b, rl && !done, akr, aki, rabs);
        bad = bad || !(rk >= T(0.1) * rabs);   // |pivot| below 0.1 of the walker's (or not finite)
      }
      inv = (int)sm[SQ::pv + 2 * N];
      const unsigned long long bm = __ballot(bad);
      if ((bm >> (lane & ~(SW - 1))) & ((1ull << SW) - 1ull)) pivoted();   // this slot: partial pivoting
    } else {
      pivoted();
    }
  }
  const T jt = slot_sum<SW>(jsum);
  if (act && sl == 0) {
    const T sg = (inv & 1) ? T(-1) : T(1);
    if (ka.logabs) ((T*)ka.logabs)[conf] = T(0.5) * lsum + jt;
    if (ka.phase) ((T*)ka.phase)[conf] = f_atan2(ui * sg, ur * sg);
  }
}

// ============================================================================================
// k_quad_grad: the Metropolis proposals of N <= 4 electrons (Be, the C atom's pseudo-valence
// electrons), value AND gradient, four configurations per wave (one 16-lane row each) --
// k_walker_rev's PROP path (walker_rev.h) restated in the row layout:
//   F1/F2/F4 as k_quad_value, keeping the conv and single-layer outputs for the backward pass;
//   F5 Phi (x) Yt and its inverse by Gauss-Jordan with partial pivoting (izamax rule, virtual
//      row exchanges, gj_inverse's arithmetic) in the row's first quad, lane c = column c;
//   B1 dL/dh^3 = Re Q_f[r,r], dL/dYt = Re(B^T (x) Phi)   (lanes 4r + f / the N^2 entries);
//   B2 back through the three layers (lane 4i + f, class sums inside the row);
//   B3 the N(N-1) pair adjoints (lane = ordered pair, forward values recomputed: 12 pairs);
//   B4 d log|psi| / d x_{e,c} on lane 4c + e from the pair adjoints and the electron-local
//      Jacobians (walker cache, or the moved electron's record).
// Outputs as the proposal path: log|psi|, |grad|^2, the moved electron's own gradient (and
// the full gradient / phase when asked).
template <typename T, int N, int A, bool WALK = false>
struct SmemQG {
  static constexpr int D0 = 4 * A;
  static constexpr int NI = QSlot<N>::NI, SW = QSlot<N>::SW;   // electron slots, lanes per configuration
  static constexpr int QM = (3 * D0 + 8) / 4;    // conv outputs of layer 0
  static constexpr int QL = (3 * 4 + 8) / 4;     // conv outputs of layers 1, 2
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  static constexpr int xs = 0;                   // [3 NI] positions; then [4] old position of the moved electron
  static constexpr int xo = 3 * NI;
  static constexpr int yv = xo + 4;              // [N][N] Yt, then its adjoint
  static constexpr int hl = yv + NI * NI;        // h^0 [NI][D0], h^3 [NI][4]; then their adjoints
  static constexpr int h3 = hl + NI * D0;
  static constexpr int g2 = h3 + NI * 4;         // [3][2][N][4] pair column means, then their adjoints
  static constexpr int S = g2 + 24 * NI;         // [NI][12] new - old patch pair values (WALK: [N][N][12] all pairs); then dbar [N][N][3]
  static constexpr int cq = S + cmax(cmax(NI * 12, 3 * NI * NI), WALK ? 12 * N * N : 0);   // conv outputs [NI][QM] + [2][NI][QL]
  static constexpr int sv = cq + NI * QM + 2 * NI * QL;      // [3][NI][4] single outputs
  static constexpr int ph = sv + 12 * NI;        // [N][N][2] Phi
  static constexpr int mx = ph + 2 * NI * NI;    // [N][N][2] B = A^{-1}
  static constexpr int size = mx + 2 * NI * NI;
  static constexpr int cqo(int l, int i) { return l == 0 ? i * QM : NI * QM + ((l - 1) * NI + i) * QL; }
};

// WALK = true: the walker launch of a sweep (k_walker_rev's walker path): the previous sweep's
// acceptance (fused), every electron's stage on lane 4c + e (its local Jacobians stay in the
// lane's registers for B4), the full pair stream on lane k N + i, and the complete walker cache
// (WCache, including the pair tanh's and the pivot record the one-wave proposal path reads).
// 5 <= N <= 8 (round 4; the C atom all-electron (6, 1), C2 (8, 2) -- the reference's example/C2):
// the proposals two configurations per wave, one 32-lane slot each, with the same phases: the
// spin-group class sums take one lane exchange across the slot's two 16-lane rows, the Gauss-Jordan
// holds two matrix elements per lane (lane 4 r + g: columns g and g + 4 of row r; the pivot is the
// packed-key max over the slot's eight row quads, as k_quad_value's LU), B3 runs the N (N - 1)
// pairs in two passes of 32, and B4 puts direction x_{e,c} on lane 8 c + e.  WALK for these shapes
// (round 4, second session): the walker launches two per wave as well -- F1's electron stage on
// lane 8 c + e (B4's lane, so the local Jacobians stay in registers), the N^2 pair stream in two
// passes of 32 lanes into a [N][N][12] block, and the pivot record written by the two-element
// Gauss-Jordan.
template <typename T, int N, int A, bool WALK = false>
__global__ __launch_bounds__(64) void k_quad_grad(KArgs ka) {
  static_assert(N <= 8, "k_quad_grad: several configurations per wave need N <= 8");
  using Ly = Lay<N, A>;
  using WC = WCache<N, A>;
  using EC = ECache<N, A>;
  using SQ = SmemQG<T, N, A, WALK>;
  constexpr int D0 = 4 * A;
  constexpr int QM = SQ::QM;
  constexpr int SW = QSlot<N>::SW, NI = QSlot<N>::NI, NSL = QSlot<N>::NSL;
  const cptr<T> P = param_ptr<T>(ka.prm);
  __shared__ T smq[NSL * SQ::size];
  const int lane = threadIdx.x;
  const int slot = lane / SW, sl = lane % SW;
  const int c0 = xcd_major(blockIdx.x, gridDim.x) * NSL + slot;
  const bool act = c0 < ka.nconf;
  const int conf = act ? c0 : ka.nconf - 1;
  T* sm = smq + slot * SQ::size;
  T* xs = sm + SQ::xs;
  T* Yv = sm + SQ::yv;
  T* hl = sm + SQ::hl;
  T* H3 = sm + SQ::h3;
  T* g2 = sm + SQ::g2;
  T* S = sm + SQ::S;
  T* cqv = sm + SQ::cq;
  T* svv = sm + SQ::sv;
  T* Ph = sm + SQ::ph;
  T* Mx = sm + SQ::mx;
  const int mper = ka.mper ? ka.mper : N, mdiv = ka.mdiv ? ka.mdiv : 1;
  const int pb = WALK ? conf : conf / mper, pi = WALK ? -1 : (conf - pb * mper) / mdiv;
  const int nup = ka.nup;
  const int* rowsrc = ka.rowsrc;
  const T RSQ2 = T(0.70710678118654752);
  const T ginv0 = T(1) / T(nup), ginv1 = T(1) / T(N - nup);
  T* Wc = (T*)ka.wcache + (size_t)pb * WC::size;
  const T* Eq = WALK ? nullptr : (const T*)ka.ecache + (size_t)conf * EC::size;
  T lv[N + D0];      // WALK: d(Yt row e, ae features of e) / d x_{e,c} of lane NI c + e
  T jd1w = T(0);     // WALK: d J_ae / d x_{e,c}
  T jsum = T(0);
  if constexpr (WALK) {
    // ---------------------------------------------------------------- F0 positions (+ acceptance)
    if (ka.acc.lpn) {
      const T te1 = taueff_wave<T>(ka.acc.taueff, ka.acc.tacc, 0, ka.acc.tstep, ka.acc.tpart);
      const T te2 = taueff_wave<T>(ka.acc.taueff, ka.acc.tacc, 1, ka.acc.tstep, ka.acc.tpart);
      if (sl < N) {   // the previous sweep's acceptance of this walker's N proposals
        T xn[3];
        const bool acc = accept_one<T, N>(ka.acc, (const T*)ka.pos, conf, sl, xn, te1, te2);
#pragma unroll
        for (int c = 0; c < 3; ++c) xs[3 * sl + c] = xn[c];
        if (acc && act) {
#pragma unroll
          for (int c = 0; c < 3; ++c) ((T*)ka.pos)[(size_t)conf * 3 * N + 3 * sl + c] = xn[c];
          if (ka.acc.count) atomicAdd(&ka.acc.count[conf], 1);
        }
      }
    } else if (sl < 3 * N) {
      xs[sl] = ((const T*)ka.pos)[(size_t)conf * 3 * N + sl];
    }
    wave_sync();
    // ---------------------------------------------------------------- F1 electron stage, lane NI c + e
    {
      const int c = sl / NI, e = sl % NI;
      const int ee = e < N ? e : N - 1;
      const bool elive = e < N, ev = c == 3;
      ElecOut<T, A> eo;
      electron_stage<T, N, A>(P, xs + ee * 3, ee, c, eo);
      T* Wl = Wc + WC::loc + 16 * (ev ? 0 : c) + ee;
#pragma unroll
      for (int col = 0; col < N; ++col) {
        PJ<T> sy = P[Ly::wy + col] * eo.yst[0];
#pragma unroll
        for (int m = 1; m < NYW; ++m) sy = sy + P[Ly::wy + m * N + col] * eo.yst[m];
        const PJ<T> yt = eo.env * sy;
        lv[col] = yt.d1;
        if (elive && ev) {
          Yv[e * N + col] = yt.v;
          if (act) Wc[WC::yv + e * N + col] = yt.v;
        }
        if (elive && !ev && act) Wl[col * 48] = yt.d1;
      }
#pragma unroll
      for (int m = 0; m < D0; ++m) {
        lv[N + m] = eo.hf[m].d1;
        if (elive && ev) {
          hl[e * D0 + m] = eo.hf[m].v;
          if (act) Wc[WC::h0 + e * D0 + m] = eo.hf[m].v;
        }
        if (elive && !ev && act) Wl[(N + m) * 48] = eo.hf[m].d1;
      }
      if (elive && ev) {
        jsum = eo.jae.v;
        if (act) Wc[WC::jaev + e] = eo.jae.v;
      }
      if (elive && !ev) {
        jd1w = eo.jae.d1;
        if (act) Wc[WC::jaed + 16 * c + e] = jd1w;
      }
    }
    // ---------------------------------------------------------------- F2 pair stream, lane k N + i
    // (N^2 > SW: passes of SW pairs)
    T jl = T(0);
#pragma unroll
    for (int it0 = 0; it0 < N * N; it0 += SW) {
      const int it = it0 + sl;
      const bool pl = it < N * N;
      const int k = pl ? it / N : 0, i = pl ? it - (it / N) * N : 0;
      const bool diag = k == i;
      T d[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) d[c] = xs[i * 3 + c] - xs[k * 3 + c];
      const T r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
      const T r = f_sqrt(diag ? T(1) : r2);
      T pp[4] = {diag ? T(0) : r, diag ? T(0) : d[0], diag ? T(0) : d[1], diag ? T(0) : d[2]};
      if (pl && k < i) {   // Pade e-e Jastrow, each pair once (Jastrow.py:51-52)
        const T cusp = P[Ly::jee_c + k * N + i], al = P[Ly::jee_a + k * N + i];
        jl += f_div(cusp * r, al * r + T(1));
      }
      if (pl) {
#pragma unroll
        for (int f = 0; f < 4; ++f) S[it * 12 + f] = pp[f];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const cptr<T> dw = P + (j == 0 ? Ly::dbl_w0 : Ly::dbl_w1);
        const cptr<T> db = P + (j == 0 ? Ly::dbl_b0 : Ly::dbl_b1);
        T q[4];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          T z = db[o];
#pragma unroll
          for (int m = 0; m < 4; ++m) z += pp[m] * dw[m * 4 + o];
          q[o] = f_tanh(z);
        }
        if (pl && !diag && act) {   // walker cache: t_{j+1} of pair (k, i) (the one-wave proposal path)
#pragma unroll
          for (int o = 0; o < 4; ++o) Wc[WC::pt + (k * N + i) * 8 + j * 4 + o] = q[o];
        }
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          pp[o] = (pp[o] + q[o]) * RSQ2;
          if (pl) S[it * 12 + (j + 1) * 4 + o] = pp[o];
        }
      }
    }
    {
      jsum += jl;
      const T jee = slot_sum<SW>(jl);
      if (sl == 0 && act) Wc[WC::jee] = jee;
    }
    wave_sync();
    // spin-group column means g2[l][G][i][f] = sum_{k in G} h2^l[k, i][f] / |G| (nn.py:151)
    for (int t = sl; t < 24 * N; t += SW) {
      const int f = t & 3, ci = (t >> 2) % N, lg = (t >> 2) / N;
      const int l = lg >> 1, G = lg & 1;
      const int k0 = G ? nup : 0, k1 = G ? N : nup;
      T acc = T(0);
      for (int k = k0; k < k1; ++k) acc += S[(k * N + ci) * 12 + l * 4 + f];
      const T v = acc * (G ? ginv1 : ginv0);
      g2[((l * 2 + G) * N + ci) * 4 + f] = v;
      if (act) Wc[WC::g2 + ((l * 2 + G) * N + ci) * 4 + f] = v;
    }
    wave_sync();
  } else {
  // ---------------------------------------------------------------- F1 cached stage of walker pb
  jsum = quad_stage_load<T, N, A, SW>((const T*)ka.pos + (size_t)pb * 3 * N, Wc, Eq, pi, sl, xs, sm + SQ::xo, Yv,
                                      hl, g2);
  wave_sync();

  // ---------------------------------------------------------------- F2 pairs of the moved electron
  {
    const int part = sl / NI, o = sl % NI;
    const int os = o < N ? o : N - 1;
    const T* xp = (part & 1) ? sm + SQ::xo : xs + pi * 3;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = part < 2 ? xs[os * 3 + c] - xp[c] : xp[c] - xs[os * 3 + c];
    T v[3][4];
    pair_values<T, N, A>(d, P, v);
    T dv[3][4];   // new - old (k_quad_value's F2)
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int f = 0; f < 4; ++f) dv[l][f] = v[l][f] - dpp<0x100 + NI>(v[l][f]);
    if (part < 2 && o < N && o != pi) {
      const T cusp = P[Ly::jee_c + pi * N + o], al = P[Ly::jee_a + pi * N + o];
      const T je = f_div(cusp * v[0][0], al * v[0][0] + T(1));
      jsum += part == 0 ? je : -je;
    }
    if (part == 0 && o < N && o != pi) {
      const int Gp = pi >= nup ? 1 : 0;
      const T gw = Gp ? ginv1 : ginv0;
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int f = 0; f < 4; ++f) g2[((l * 2 + Gp) * N + o) * 4 + f] += dv[l][f] * gw;
    }
    if (part == 2) {
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int f = 0; f < 4; ++f) S[o * 12 + l * 4 + f] = dv[l][f];
    }
  }
  wave_sync();
#pragma unroll
  for (int t0 = 0; t0 < 24; t0 += SW) {
    const int t = t0 + sl;
    if (t < 24) {
      const int l = t >> 3, G = (t >> 2) & 1, f = t & 3;
      const int k0 = G ? nup : 0, k1 = G ? N : nup;
      T acc = T(0);
      for (int k = k0; k < k1; ++k)
        if (k != pi) acc += S[k * 12 + l * 4 + f];
      g2[((l * 2 + G) * N + pi) * 4 + f] += acc * (G ? ginv1 : ginv0);
    }
  }
  wave_sync();
  }   // proposal path

  // ---------------------------------------------------------------- F4 h-stream layers (values kept)
  const int fi = sl >> 2, ff = sl & 3;
  const bool ilive = fi < N;
  const int ic = ilive ? fi : N - 1;
  const bool inG1 = ic >= nup;
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
        gown[0][t] = slot_class4_sum<SW>(inG1 ? T(0) : x) * ginv0;
        gown[1][t] = slot_class4_sum<SW>(inG1 ? x : T(0)) * ginv1;
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
        if (ilive) cqv[SQ::cqo(l, ic) + q0 + ff] = c;
        cq[q0 + 0] = quad_bcast<0>(c);
        cq[q0 + 1] = quad_bcast<1>(c);
        cq[q0 + 2] = quad_bcast<2>(c);
        cq[q0 + 3] = quad_bcast<3>(c);
      }
    }
#pragma unroll
    for (int q = 0; q < QM; ++q)
      if (q >= 4 * QF && q < Q) {
        cq[q] = f_tanh(zc[q] * T(0.25) + convb[q]);
        if (ilive && (q & 3) == ff) cqv[SQ::cqo(l, ic) + q] = cq[q];
      }
    T z = sngb[ff], z1 = T(0);
#pragma unroll
    for (int q = 0; q < QM; ++q)
      if (q < Q) {
        if (q & 1) z1 += cq[q] * sngw[q * 4 + ff];
        else z += cq[q] * sngw[q * 4 + ff];
      }
    z += z1;
    const T sval = f_tanh(z);
    if (ilive) svv[(l * NI + ic) * 4 + ff] = sval;
    const T hin = l == 0 ? hl[ic * D0 + ff] : hreg;
    hreg = (d1 == NH) ? (hin + sval) * RSQ2 : sval;
  }
  if (ilive) H3[ic * 4 + ff] = hreg;
  wave_sync();

  // ---------------------------------------------------------------- F5 Phi, A = Phi (x) Yt, B = A^{-1}
  // one matrix element per lane (lane 4r + c of the row holds A[r][c]); in-place Gauss-Jordan with
  // virtual partial pivoting (gj_inverse's steps): after step k the pivot row p_k holds
  // q = row / pivot (q_k = 1 / pivot), every other row r has a[r][c] - a[r][k] q_c (column k:
  // -a[r][k] q_k); then B[k][p_c] = X[p_k][c].  The pivot row of column k is the max of packed keys
  // (|re| + |im| bits, low bits 3 - r) over the column's lanes by two DPP row rotations among the
  // rows not used yet.
  T lsum = T(0), ur = T(1), ui = T(0);
  int inv = 0;
  if constexpr (SW == 16) {
    const int r = sl >> 2, c = sl & 3;
    const bool rl = r < N;
    T a = T(0), b = T(0);
    if (rl && c < N) {
      const int src = rowsrc[r];
      const int sp = r < nup ? 0 : 1;
      T re = P[Ly::orb_b + (sp * N + c) * 2 + 0], im = P[Ly::orb_b + (sp * N + c) * 2 + 1];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const T hv = H3[src * 4 + f];
        re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 0];
        im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1];
      }
      Ph[(r * N + c) * 2 + 0] = re;
      Ph[(r * N + c) * 2 + 1] = im;
      const T y = Yv[r * N + c];
      a = re * y;
      b = im * y;
    }
    const int rowbase = lane & ~15;
    unsigned used = 0;
    int stepk = 0;   // the step at which this lane's row was the pivot row
    int pc = 0;      // the pivot row of step c (this lane's column)
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const T akr = k == 0 ? quad_bcast<0>(a) : (k == 1 ? quad_bcast<1>(a) : (k == 2 ? quad_bcast<2>(a) : quad_bcast<3>(a)));
      const T aki = k == 0 ? quad_bcast<0>(b) : (k == 1 ? quad_bcast<1>(b) : (k == 2 ? quad_bcast<2>(b) : quad_bcast<3>(b)));
      const bool open = rl && !((used >> r) & 1u);
      unsigned key = open ? ((key_bits(f_abs(akr) + f_abs(aki)) & ~3u) | (unsigned)(3 - r)) : 0u;
      {
        const unsigned k4 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x124, 0xF, 0xF, true);
        key = key > k4 ? key : k4;
        const unsigned k8 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x128, 0xF, 0xF, true);
        key = key > k8 ? key : k8;
      }
      const int p = 3 - (int)(key & 3u);
      const T p0r = row_bcast(a, k), p1r = row_bcast(a, 4 + k), p2r = row_bcast(a, 8 + k), p3r = row_bcast(a, 12 + k);
      const T p0i = row_bcast(b, k), p1i = row_bcast(b, 4 + k), p2i = row_bcast(b, 8 + k), p3i = row_bcast(b, 12 + k);
      const T pr = p == 0 ? p0r : (p == 1 ? p1r : (p == 2 ? p2r : p3r));
      const T pim = p == 0 ? p0i : (p == 1 ? p1i : (p == 2 ? p2i : p3i));
      const T spr = __shfl(a, rowbase + 4 * p + c), spi = __shfl(b, rowbase + 4 * p + c);   // A[p][c]
      inv += __builtin_popcount(used >> p);
      used |= 1u << p;
      const T den = pr * pr + pim * pim;
      T ipr_, ipi_, rabs_, lden_;
      pivot_recip(pr, pim, den, ipr_, ipi_, rabs_, lden_);
      lsum += lden_;
      {
        const T rm = rabs_;
        const T xr = pr * rm, xi = pim * rm;
        const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
        ur = nr;
        ui = ni;
      }
      if (WALK && sl == 0 && act) {   // pivot record (gj.h: row of step k, 1 / |pivot_k|)
        Wc[WC::pv + k] = T(p);
        Wc[WC::pv + N + k] = rabs_;
        Wc[WC::pv + 2 * N + 2 + k] = rabs_;
      }
      const T ir = ipr_, ii = ipi_;   // 1 / pivot
      const bool ck = (c == k);
      const T qr = ck ? ir : spr * ir - spi * ii;
      const T qi = ck ? ii : spr * ii + spi * ir;
      const T br = ck ? T(0) : a, bi = ck ? T(0) : b;
      const T nr = br - (akr * qr - aki * qi);
      const T ni = bi - (akr * qi + aki * qr);
      a = r == p ? qr : nr;
      b = r == p ? qi : ni;
      stepk = r == p ? k : stepk;
      pc = ck ? p : pc;
    }
    if (rl && c < N) {
      Mx[(stepk * N + pc) * 2 + 0] = a;
      Mx[(stepk * N + pc) * 2 + 1] = b;
    }
    if (WALK && sl == 0 && act) {
      Wc[WC::pv + 2 * N] = T(inv & 1);
      Wc[WC::pv + 2 * N + 1] = T(0.5) * lsum;
    }
  } else {
    // 5 <= N <= 8: lane 4 r + g of the slot holds A[r][g] and A[r][g + 4].  Step k: column k
    // reaches row r's lanes by a quad broadcast, the pivot row p is the packed-key max over the
    // slot's eight row quads (low three bits 7 - r: the first maximal row, izamax, as gj.h), the
    // pivot row's entries of this lane's two columns come by lane permutes; then, as above,
    // q = A[p][:] / pivot (q_k = 1 / pivot), A[r][c] -= A[r][k] q_c for r != p (column k:
    // -A[r][k] q_k), row p <- q.  B[k][p_c] = X[p_k][c].
    const int r = sl >> 2, g = sl & 3;
    const bool rl = r < N;
    T a[2], b[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = g + 4 * h;
      a[h] = T(0);
      b[h] = T(0);
      if (rl && c < N) {
        const int src = rowsrc[r];
        const int sp = r < nup ? 0 : 1;
        T re = P[Ly::orb_b + (sp * N + c) * 2 + 0], im = P[Ly::orb_b + (sp * N + c) * 2 + 1];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const T hv = H3[src * 4 + f];
          re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 0];
          im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1];
        }
        Ph[(r * N + c) * 2 + 0] = re;
        Ph[(r * N + c) * 2 + 1] = im;
        const T y = Yv[r * N + c];
        a[h] = re * y;
        b[h] = im * y;
      }
    }
    const int sbase = lane & ~31;
    unsigned used = 0;
    int stepk = 0;      // the step at which this lane's row was the pivot row
    int pc[2] = {0, 0};   // the pivot row of step c for this lane's two columns
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int kh = k >> 2;
      T akr, aki;   // A[r][k]
      if ((k & 3) == 0) { akr = quad_bcast<0>(a[kh]); aki = quad_bcast<0>(b[kh]); }
      else if ((k & 3) == 1) { akr = quad_bcast<1>(a[kh]); aki = quad_bcast<1>(b[kh]); }
      else if ((k & 3) == 2) { akr = quad_bcast<2>(a[kh]); aki = quad_bcast<2>(b[kh]); }
      else { akr = quad_bcast<3>(a[kh]); aki = quad_bcast<3>(b[kh]); }
      const bool open = rl && !((used >> r) & 1u);
      unsigned key = open ? ((key_bits(f_abs(akr) + f_abs(aki)) & ~7u) | (unsigned)(7 - r)) : 0u;
      {
        const unsigned k4 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x124, 0xF, 0xF, true);
        key = key > k4 ? key : k4;
        const unsigned k8 = (unsigned)__builtin_amdgcn_mov_dpp((int)key, 0x128, 0xF, 0xF, true);
        key = key > k8 ? key : k8;
        const unsigned k16 = (unsigned)__shfl_xor((int)key, 16);
        key = key > k16 ? key : k16;
      }
      const int p = 7 - (int)(key & 7u);
      const int srcl = sbase + 4 * p + g;
      T er[2], ei[2];   // A[p][g], A[p][g + 4]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        er[h] = __shfl(a[h], srcl);
        ei[h] = __shfl(b[h], srcl);
      }
      T pr, pim;   // A[p][k]
      {
        const T sr = er[kh], si = ei[kh];
        if ((k & 3) == 0) { pr = quad_bcast<0>(sr); pim = quad_bcast<0>(si); }
        else if ((k & 3) == 1) { pr = quad_bcast<1>(sr); pim = quad_bcast<1>(si); }
        else if ((k & 3) == 2) { pr = quad_bcast<2>(sr); pim = quad_bcast<2>(si); }
        else { pr = quad_bcast<3>(sr); pim = quad_bcast<3>(si); }
      }
      inv += __builtin_popcount(used >> p);
      used |= 1u << p;
      const T den = pr * pr + pim * pim;
      T ipr_, ipi_, rabs_, lden_;
      pivot_recip(pr, pim, den, ipr_, ipi_, rabs_, lden_);
      lsum += lden_;
      {
        const T rm = rabs_;
        const T xr = pr * rm, xi = pim * rm;
        const T nr = ur * xr - ui * xi, ni = ur * xi + ui * xr;
        ur = nr;
        ui = ni;
      }
      if (WALK && sl == 0 && act) {   // pivot record (gj.h: row of step k, 1 / |pivot_k|)
        Wc[WC::pv + k] = T(p);
        Wc[WC::pv + N + k] = rabs_;
        Wc[WC::pv + 2 * N + 2 + k] = rabs_;
      }
      const T ir = ipr_, ii = ipi_;   // 1 / pivot
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool ck = (g + 4 * h == k);
        const T qr = ck ? ir : er[h] * ir - ei[h] * ii;
        const T qi = ck ? ii : er[h] * ii + ei[h] * ir;
        const T br = ck ? T(0) : a[h], bi = ck ? T(0) : b[h];
        const T nr = br - (akr * qr - aki * qi);
        const T ni = bi - (akr * qi + aki * qr);
        a[h] = r == p ? qr : nr;
        b[h] = r == p ? qi : ni;
        pc[h] = ck ? p : pc[h];
      }
      stepk = r == p ? k : stepk;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = g + 4 * h;
      if (rl && c < N) {
        Mx[(stepk * N + pc[h]) * 2 + 0] = a[h];
        Mx[(stepk * N + pc[h]) * 2 + 1] = b[h];
      }
    }
    if (WALK && sl == 0 && act) {
      Wc[WC::pv + 2 * N] = T(inv & 1);
      Wc[WC::pv + 2 * N + 1] = T(0.5) * lsum;
    }
  }
  wave_sync();
#define BRE(c, s) Mx[((c) * N + (s)) * 2]
#define BIM(c, s) Mx[((c) * N + (s)) * 2 + 1]

  // ---------------------------------------------------------------- B1 adjoints of h^3 and Yt
  T* hbar = hl;   // h^0 / h^3 are dead from here: their adjoints take their places
  if (sl < 4 * N) {
    const int r = sl >> 2, f = sl & 3;
    const int sp = r < nup ? 0 : 1;
    T q = T(0);
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const T yv = Yv[r * N + c];
      const T wr = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2] * yv;
      const T wi = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1] * yv;
      q += wr * BRE(c, r) - wi * BIM(c, r);
    }
    H3[rowsrc[r] * 4 + f] = q;   // adjoint of h^3 (same place)
  }
  wave_sync();   // ybar overwrites Yt
#pragma unroll
  for (int e0 = 0; e0 < N * N; e0 += SW) {
    const int e = e0 + sl;
    if (e < N * N) {
      const int r = e / N, c = e - r * N;
      Yv[e] = BRE(c, r) * Ph[e * 2] - BIM(c, r) * Ph[e * 2 + 1];
    }
  }
#undef BRE
#undef BIM
  wave_sync();

  // ---------------------------------------------------------------- B2 back through the layers
  T* g2b = g2;   // the g2 values are dead after F4
  {
    T hb = H3[ic * 4 + ff];
#pragma unroll
    for (int l = 2; l >= 0; --l) {
      const int d1 = l == 0 ? D0 : NH;
      const int DF = 3 * d1 + 8;
      const int Q = DF / 4;
      const int T4 = d1 / 4;
      const cptr<T> convw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2)) + ic * DF;
      const cptr<T> sngw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
      const T sval = svv[(l * NI + ic) * 4 + ff];
      const T sb = (d1 == NH) ? hb * RSQ2 : hb;
      const T zs = sb * (T(1) - sval * sval);
      const T zq[4] = {quad_bcast<0>(zs), quad_bcast<1>(zs), quad_bcast<2>(zs), quad_bcast<3>(zs)};
      const int QF = Q / 4;
      T cg[QM];
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const bool full = q < 4 * QF;
        if (q < Q && (!full || (q & 3) == 0)) {
          const int qq = full ? q + ff : q;
          T cb = T(0);
#pragma unroll
          for (int m = 0; m < 4; ++m) cb += zq[m] * sngw[qq * 4 + m];
          const T c = cqv[SQ::cqo(l, ic) + qq];
          const T g = cb * (T(1) - c * c) * T(0.25);
          if (full) {
            cg[q + 0] = quad_bcast<0>(g);
            cg[q + 1] = quad_bcast<1>(g);
            cg[q + 2] = quad_bcast<2>(g);
            cg[q + 3] = quad_bcast<3>(g);
          } else {
            cg[q] = g;
          }
        }
      }
      T fb[QM];
#pragma unroll
      for (int q = 0; q < QM; ++q)
        if (q < Q) fb[q] = cg[q] * convw[4 * q + ff];
      if (ilive) {   // pre-scaled by the group-mean weights 1/|G| of the pair sums
        g2b[((l * 2 + 0) * N + ic) * 4 + ff] = fb[3 * T4 + 0] * ginv0;
        g2b[((l * 2 + 1) * N + ic) * 4 + ff] = fb[3 * T4 + 1] * ginv1;
      }
      T hn = T(0);
#pragma unroll
      for (int t = 0; t < D0 / 4; ++t) {
        if (t < T4) {
          const T s0 = slot_class4_sum<SW>(ilive ? fb[T4 + t] : T(0)) * ginv0;
          const T s1 = slot_class4_sum<SW>(ilive ? fb[2 * T4 + t] : T(0)) * ginv1;
          T v = fb[t] + (inG1 ? s1 : s0);
          if (d1 == NH) v += hb * RSQ2;
          if (l == 0) {
            if (ilive) hbar[ic * D0 + ff + 4 * t] = v;
          } else {
            hn = v;
          }
        }
      }
      hb = hn;
    }
  }
  wave_sync();

  // ---------------------------------------------------------------- B3 pair adjoints (every pair fresh)
  T* dbar = S;   // [N][N][3]
#pragma unroll
  for (int it0 = 0; it0 < N * (N - 1); it0 += SW) {
  const int it = it0 + sl;
  if (it < N * (N - 1)) {
    const int k = it / (N - 1), jj = it - k * (N - 1);
    const int i = jj + (jj >= k ? 1 : 0);
    const int G = k >= nup ? 1 : 0;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = xs[i * 3 + c] - xs[k * 3 + c];
    const T r = f_sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    const T p0[4] = {r, d[0], d[1], d[2]};
    T t1[4], p1[4], t2[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      T s = P[Ly::dbl_b0 + o];
#pragma unroll
      for (int m = 0; m < 4; ++m) s += p0[m] * P[Ly::dbl_w0 + m * 4 + o];
      t1[o] = f_tanh(s);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) p1[o] = (p0[o] + t1[o]) * RSQ2;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      T s = P[Ly::dbl_b1 + o];
#pragma unroll
      for (int m = 0; m < 4; ++m) s += p1[m] * P[Ly::dbl_w1 + m * 4 + o];
      t2[o] = f_tanh(s);
    }
    T pb2[4], pb1[4], pb0[4], z2[4], z1[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) pb2[f] = g2b[((2 * 2 + G) * N + i) * 4 + f];
#pragma unroll
    for (int o = 0; o < 4; ++o) z2[o] = pb2[o] * RSQ2 * (T(1) - t2[o] * t2[o]);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T s = g2b[((1 * 2 + G) * N + i) * 4 + m] + pb2[m] * RSQ2;
#pragma unroll
      for (int o = 0; o < 4; ++o) s += z2[o] * P[Ly::dbl_w1 + m * 4 + o];
      pb1[m] = s;
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) z1[o] = pb1[o] * RSQ2 * (T(1) - t1[o] * t1[o]);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T s = g2b[((0 * 2 + G) * N + i) * 4 + m] + pb1[m] * RSQ2;
#pragma unroll
      for (int o = 0; o < 4; ++o) s += z1[o] * P[Ly::dbl_w0 + m * 4 + o];
      pb0[m] = s;
    }
    T rb = pb0[0];
    if (k < i) {   // Pade e-e Jastrow once per unordered pair
      const T cusp = P[Ly::jee_c + k * N + i], al = P[Ly::jee_a + k * N + i];
      const T den = al * r + T(1);
      rb += cusp * f_rcp(den * den);
    }
    const T ir = f_rcp(r);
#pragma unroll
    for (int c = 0; c < 3; ++c) dbar[(k * N + i) * 3 + c] = pb0[1 + c] + rb * d[c] * ir;
  }
  }
  wave_sync();

  // ---------------------------------------------------------------- B4 gradient, lane NI c + e
  const int gc = sl / NI, ge = sl % NI;
  const bool gdir = gc < 3 && ge < N;
  const int gcc = gc < 3 ? gc : 0, gee = ge < N ? ge : N - 1;
  T g = T(0);
  if constexpr (WALK) {
    // lane NI c + e: the same lane as in F1, whose local Jacobians are in registers
    g = jd1w;
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k != gee) g += dbar[(k * N + gee) * 3 + gcc] - dbar[(gee * N + k) * 3 + gcc];
#pragma unroll
    for (int col = 0; col < N; ++col) g = f_fma(Yv[gee * N + col], lv[col], g);
#pragma unroll
    for (int m = 0; m < D0; ++m) g = f_fma(hbar[gee * D0 + m], lv[N + m], g);
  } else {
    const bool mov = gee == pi;
    const int l64 = 16 * gcc + gee;   // the walker cache's direction-lane index
    T jd = Wc[WC::jaed + l64];
    if (mov) jd = Eq[EC::jd + gcc];
    g = jd;
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k != gee) g += dbar[(k * N + gee) * 3 + gcc] - dbar[(gee * N + k) * 3 + gcc];
#pragma unroll
    for (int col = 0; col < N; ++col) {
      const T lw = mov ? Eq[EC::yd + gcc * N + col] : Wc[WC::loc + col * 48 + l64];
      g = f_fma(Yv[gee * N + col], lw, g);
    }
#pragma unroll
    for (int m = 0; m < D0; ++m) {
      const T lw = mov ? Eq[EC::hd + gcc * D0 + m] : Wc[WC::loc + (N + m) * 48 + l64];
      g = f_fma(hbar[gee * D0 + m], lw, g);
    }
  }
  const T gd = gdir ? g : T(0);
  const T sumsq = slot_sum<SW>(gd * gd);
  const T jt = slot_sum<SW>(jsum);
  const T lsum0 = quad_bcast<0>(lsum), ur0 = quad_bcast<0>(ur), ui0 = quad_bcast<0>(ui);
  if (act) {
    if (ka.grad && gdir) ((T*)ka.grad)[(size_t)conf * 3 * N + 3 * gee + gcc] = g;
    if (ka.gown && gdir && gee == pi) ((T*)ka.gown)[(size_t)conf * 3 + gcc] = g;
    if (sl == 0) {
      const T sg = (inv & 1) ? T(-1) : T(1);
      if (ka.logabs) ((T*)ka.logabs)[conf] = T(0.5) * lsum0 + jt;
      if (ka.phase) ((T*)ka.phase)[conf] = f_atan2(ui0 * sg, ur0 * sg);
      if (ka.sumsq) ((T*)ka.sumsq)[conf] = sumsq;
      if (ka.tacc) tacc_add(ka.tacc, WALK ? 0 : 1, conf, (double)sumsq);
    }
    if (WALK && ka.dg1 && sl < N) {   // the sweep's draws of walker conf (k_draws' arithmetic)
      const uint32_t t = (uint32_t)(conf * N + sl);
      float a[3], b[3], c[4];
      philox_normal3f(ka.seed, ka.step, t, 0u, a);
      philox_normal3f(ka.seed, ka.step, t, 1u, b);
      philox_u4(ka.seed, ka.step, t, 2u, c);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        ((T*)ka.dg1)[(size_t)t * 3 + k] = (T)a[k];
        ((T*)ka.dg2)[(size_t)t * 3 + k] = (T)b[k];
      }
      ((T*)ka.du)[t] = (T)(c[0] - 5.9604644775390625e-08f);
    }
  }
}

}  // namespace aq
