// walker_lap.h -- local energy E_L = V - (lap log|psi| + |grad log|psi||^2) / 2 of the AIQMC
// wavefunction (Energy/hamiltonian.py:236-260, complex_output=False; the reference's
// jvp-of-grad loop :100-131) in two launches, one wavefront per walker each.
//
// 1. k_walker_rev<T,N,A,PREP=true> (walker_rev.h): the reverse-mode kernel's value pass
//    and its adjoint pass through the mean-field (h) stream; writes the walker's
//    LapCache (layout.h): for every tanh node m of the h stream its derivative 1 - t^2 and
//    its curvature weight abar_m phi''(z_m) (abar = d log|det A| / d node, phi'' =
//    -2 t (1 - t^2)); the adjoints of the layer-0 features; the pair-stream derivative
//    sums sd; B = A^{-1}, Phi, Q_f = P_f B; and the pair-local part of the Laplacian.
//
// 2. k_walker_lap<T,N,A> (this file) carries FIRST derivatives only, lane (c, e) = the
//    direction x_{e,c} (jets.h layout).  Every h-stream node is tanh of a linear map, so
//    the determinant's term sum_{r,f} Hbar[r,f] lap H[r,f] (Hbar = Re Q_f[r,r]) equals
//        sum_m abar_m phi''(z_m) |grad z_m|^2  +  sum_leaves abar_leaf lap(leaf)
//    (leaves: the ae features, the pair terms of the column means g2).  Each direction
//    lane adds abar_m phi''(z_m) (dz_m/dx_{e,c})^2 per node; no lane carries second
//    derivatives through the dense stream (the forward-Laplacian kernel walker_kernel.h
//    does, with twice the per-lane state and one wave per SIMD).  The determinant's own
//    second-order terms use its low-rank structure (walker_kernel.h header):
//        Re[(2 dPhi_e.Yt' + Phi_e.Yt'') b_e - sum_{r,s} S_rs S_sr - 2 sum_r z_r S_re - (w.b_e)^2]
//    with S = sum_f diag(U_f) Q_f, U = dH/dx_{e,c}, w = Phi[e,:] dYt[e,:], z = B^T w.  The
//    Jastrow factors and the per-electron stage (envelope, Ylm stream, ae features) are
//    second-order jets along the lane direction.
#pragma once
#include "electron.h"
#include "jets.h"
#include "layout.h"
#include "walker_kernel.h"
#include "walker_rev.h"

namespace aq {

// Diagnostics build (-DAQ_PHASE_PROF): per-phase shader-clock cycles of k_walker_lap, summed over waves
// into aq_phase_cycles[16 + k] (the proposal slots: no proposal runs inside a local-energy call; the
// adjoint pass records into [0..9])
#ifdef AQ_PHASE_PROF
#define LPH(k)                                                                            \
  do {                                                                                    \
    const unsigned long long t_ = __builtin_readcyclecounter();                           \
    if ((threadIdx.x & 63) == 0) atomicAdd(&aq_phase_cycles[16 + (k)], t_ - t_ph);        \
    t_ph = t_;                                                                            \
  } while (0)
#else
#define LPH(k) \
  do {         \
  } while (0)
#endif

template <typename T, int N, int A>
struct SmemLap {
  static constexpr int xs = 0;                               // [48] positions
  static constexpr int ly = 48;                              // one layer's LapCache block
  // lane-private arrays [..][49]: direction lanes 0..47 own a column; the 16 value-row
  // lanes share column 48 (they carry no derivatives; their stores there are don't-cares)
  static constexpr int yd = ly + LapCache<N, A>::layer_n;    // [2][N][49] dYt/dx, d2Yt/dx2 of row le
  static constexpr int hb = (yd + 2 * N * 49 + 3) / 4 * 4;   // [N][49][4] dh/dx (a lane's 4 units: one 16-byte access)
  static constexpr int end = hb + N * NH * 49;
  // Q_f [N][N][4][2] (and B [N][N][2] where it fits) staged over ly + yd once both are dead
  static constexpr int qs = ly;
  static constexpr int bs = qs + 8 * N * N;
  static constexpr bool stage_b = 10 * N * N <= LapCache<N, A>::layer_n + 2 * N * 49;
  static_assert(8 * N * N <= LapCache<N, A>::layer_n + 2 * N * 49, "Q_f must fit over ly + yd");
  static constexpr int bytes = ((end * (int)sizeof(T)) + 15) & ~15;
  static_assert(end - ly >= 3 * 3 * 64, "multi-wave partial sums (W <= 4) must fit behind ly");
};

// Workgroup copy of n elements of a LapCache block to LDS in 16-byte pieces (n * sizeof(T) is a
// multiple of 16 for every staged block; all offsets are 16-byte aligned): a quarter of the load
// and store instructions of an element-wise copy, and one round of loads in flight per block.
template <typename T>
__device__ __forceinline__ void stage_copy(T* dst, cptr<T> src, int n) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(4))) u4* s = (const __attribute__((address_space(4))) u4*)src;
  u4* d = (u4*)dst;
  const int cnt = n * (int)sizeof(T) / 16;
  for (int i = threadIdx.x; i < cnt; i += blockDim.x) d[i] = s[i];
  // a tail shorter than 16 bytes (odd-sized blocks; none of the built shapes has one, and with a
  // compile-time n the loop folds away)
  for (int i = cnt * 16 / (int)sizeof(T) + (int)threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// The same copy split in two, so that the loads of a block can be issued a phase ahead of the
// barrier that frees its LDS destination: stage_load issues this thread's 16-byte pieces into
// registers (NU >= the pieces per thread of a one-wave workgroup), stage_store writes them.
typedef unsigned int u4s __attribute__((ext_vector_type(4)));
template <typename T, int CNT>
struct StageRegs {
  static constexpr int PIECES = CNT * (int)sizeof(T) / 16;
  static constexpr int NU = (PIECES + 63) / 64 > 0 ? (PIECES + 63) / 64 : 1;
  static constexpr int TL = CNT - PIECES * 16 / (int)sizeof(T);   // a tail shorter than 16 bytes (odd N)
  u4s r[NU];
  T tail;
  __device__ __forceinline__ void load(cptr<T> src) {
    const __attribute__((address_space(4))) u4s* s = (const __attribute__((address_space(4))) u4s*)src;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int i = (int)threadIdx.x + k * (int)blockDim.x;
      if (i < PIECES) r[k] = s[i];
    }
    if (TL > 0 && (int)threadIdx.x < TL) tail = src[CNT - TL + (int)threadIdx.x];
  }
  __device__ __forceinline__ void store(T* dst) const {
    u4s* d = (u4s*)dst;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int i = (int)threadIdx.x + k * (int)blockDim.x;
      if (i < PIECES) d[i] = r[k];
    }
    if (TL > 0 && (int)threadIdx.x < TL) dst[CNT - TL + (int)threadIdx.x] = tail;
  }
};
// local-energy stage prefetch (round 6, interleaved A/B on one box, N2 4096 walkers, µs per E_L
// pair: 194.7 / 195.1 -> 192.2 / 191.3, E_L and positions bitwise equal;
// profiles/r06_s2_ab_lap_prefetch.txt).  -DAQ_LAP_NO_PREFETCH: the synchronous stage_copy.  Layer
// 0's block kept in registers over the per-electron stage and E2's Phi row loaded with Q_f as well:
// 190.1 / 189.4 vs 189.9 / 190.0, not bitwise (operand order); not kept (profiles/r06_s3_ab_lap_prefetch2.txt).
#ifndef AQ_LAP_NO_PREFETCH
constexpr bool kLapPrefetch = true;
#else
constexpr bool kLapPrefetch = false;
#endif

// One h-stream layer (nn.py:280-311) in first derivatives, column loop over electrons i.
// ly: this layer's LapCache block (LDS); hb: dh/dx of every electron [N][49][NH], updated in place
// (column `lane` = min(lane, 48), see SmemLap).
// One column's record of the lane's pair (le, i): layers 1, 2 take the double layers' tanh outputs t1, t2
// (LapCache pt, 16-byte chunks 0 .. NCH - 1); layer 0 (NCH = 0) the e-e Jastrow parameters cusp, alpha of
// the pair from the parameter block
template <typename T, int N, int A, int NCH>
struct PairT {
  T t[NCH > 0 ? NCH : 1][4];
  __device__ __forceinline__ void load(cptr<T> src, cptr<T> P, int le, int i) {
    if constexpr (NCH == 0) {
      using Ly = Lay<N, A>;
      t[0][0] = P[Ly::jee_c + le * N + i];
      t[0][1] = P[Ly::jee_a + le * N + i];
    } else if constexpr (sizeof(T) == 4) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      const __attribute__((address_space(4))) f4* s = (const __attribute__((address_space(4))) f4*)src;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const f4 v = s[j];
        t[j][0] = v.x;
        t[j][1] = v.y;
        t[j][2] = v.z;
        t[j][3] = v.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int o = 0; o < 4; ++o) t[j][o] = src[j * 4 + o];
    }
  }
};

template <typename T, int N, int A, int L>
__device__ __forceinline__ void lap_layer(cptr<T> P, const T* xs, T* hb, const T* ly, const PJ<T>* hf, int lane,
                                          int lc, int er, int le, bool val, bool dir, bool live, int nup, T& jd1,
                                          T& jd2, T& vv, T& acc, int wv, int W, cptr<T> Lpt) {
  using Ly = Lay<N, A>;
  using LC = LapCache<N, A>;
  constexpr int DIN = (L == 0) ? 4 * A : NH;
  constexpr int DF = 3 * DIN + 2 * NH2;
  constexpr int Q = DF / 4;
  const cptr<T> convw = P + (L == 0 ? Ly::conv_w0 : (L == 1 ? Ly::conv_w1 : Ly::conv_w2));
  const cptr<T> sngw = P + (L == 0 ? Ly::sng_w0 : (L == 1 ? Ly::sng_w1 : Ly::sng_w2));
  const T ginv[2] = {T(1) / T(nup), T(1) / T(N - nup)};
  const T RSQ2 = T(0.70710678118654752);   // residual (x + y)/sqrt(2), nn.py:284
  const bool inG[2] = {live && er < nup, live && er >= nup};
  const int c3 = lc < 3 ? lc : 0;

  // spin-group means of h (construct_symmetric_features, nn.py:142-150)
  T g1[2][DIN];
  if constexpr (L == 0) {
#pragma unroll
    for (int G = 0; G < 2; ++G)
#pragma unroll
      for (int m = 0; m < DIN; ++m) g1[G][m] = (dir && inG[G]) ? hf[m].d1 * ginv[G] : T(0);
  } else {
#pragma unroll
    for (int m = 0; m < DIN; ++m) g1[0][m] = g1[1][m] = T(0);
    for (int k = 0; k < nup; ++k)
#pragma unroll
      for (int m = 0; m < DIN; ++m) g1[0][m] += hb[(k * 49 + lane) * NH + m];
    for (int k = nup; k < N; ++k)
#pragma unroll
      for (int m = 0; m < DIN; ++m) g1[1][m] += hb[(k * 49 + lane) * NH + m];
#pragma unroll
    for (int m = 0; m < DIN; ++m) {
      g1[0][m] *= ginv[0];
      g1[1][m] *= ginv[1];
    }
    if (W > 1) __syncthreads();   // every wave has read layer L's dh/dx before any overwrites it
  }

  // multi-wave mode: wave wv of the walker's workgroup takes columns i = wv, wv + W, ...
  // Two columns per iteration (round 4, N2 4096 walkers, local-energy pair 195.9-196.6 -> 193.5-193.9 us
  // at the same 191 VGPRs; by four, or E4's (r, s) loop by two / four as well: no further gain,
  // profiles/r04_s9_ab_lap_unroll.txt)
  // the lane's pair records (le, i): layers 1, 2 the double layers' tanh outputs (LapCache pt, written by
  // the adjoint pass: the column loop carries only the derivative chain), layer 0 the e-e Jastrow
  // parameters.  Two columns per iteration, the next iteration's records loaded at its top (a whole
  // iteration of arithmetic in flight before they are used)
  using Rec = PairT<T, N, A, L>;
  constexpr int PS = LC::pt_n;
  auto column = [&](int i, const Rec& tcur) {
    const bool diag = (le == i);
    // single-node weights of column i first: read before this column's dh/dx stores (LDS, in order)
    const T* sn = ly + LC::sn + i * NH * 2;
    T snv[2 * NH];
#pragma unroll
    for (int f = 0; f < 2 * NH; ++f) snv[f] = sn[f];
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = xs[i * 3 + c] - xs[le * 3 + c];
    const T r = f_sqrt(diag ? T(1) : d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    const T ir = f_rcp(r);
    const T dl = c3 == 0 ? d[0] : (c3 == 1 ? d[1] : d[2]);
    const T r1 = -dl * ir;   // dr/dx_{le,lc}, with d = x_i - x_le
    if constexpr (L == 0) {
      // Pade e-e Jastrow term cusp r / (1 + alpha r) of pair (le, i) (Jastrow.py:51-52)
      const T cusp = tcur.t[0][0], al = tcur.t[0][1];
      const T iden = f_rcp(al * r + T(1));
      const T j1 = cusp * iden * iden;          // J'(r)
      const T j2 = T(-2) * al * j1 * iden;      // J''(r)
      if (dir && !diag) {
        jd1 += j1 * r1;
        jd2 += j2 * r1 * r1 + j1 * (T(1) - r1 * r1) * ir;
      }
      if (val && live && er < i) vv += ir;      // V_ee, each pair once (hamiltonian.py:177-187)
    }
    // pair stream h2[le,i] = [r, x_i - x_le] through L double layers (nn.py:305-309): the derivative
    // along x_{le,lc}, with the layers' tanh outputs of the adjoint pass
    T pd[4];
    pd[0] = r1;
#pragma unroll
    for (int c = 0; c < 3; ++c) pd[1 + c] = (lc == c) ? T(-1) : T(0);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const cptr<T> dw = P + (j == 0 ? Ly::dbl_w0 : Ly::dbl_w1);
      T td[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        T zd = T(0);
#pragma unroll
        for (int m = 0; m < 4; ++m) zd += pd[m] * dw[m * 4 + o];
        const T tv = tcur.t[j][o];
        td[o] = (T(1) - tv * tv) * zd;
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) pd[o] = (pd[o] + td[o]) * RSQ2;
    }
    // column means of h2 over the spin groups (nn.py:151): lane (c, e != i) sees pair (e, i)
    // only; lane (c, i) sees every pair (k, i) -- their derivative sums from the LapCache
    const T* sdp = ly + LC::sd + (i * 3 + c3) * 4;
    T g2[2][4];
#pragma unroll
    for (int G = 0; G < 2; ++G) {
      const T cP = (dir && inG[G] && !diag) ? ginv[G] : T(0);
      const T cS = (dir && diag) ? ginv[G] : T(0);
#pragma unroll
      for (int f = 0; f < 4; ++f) g2[G][f] = cP * pd[f] + cS * sdp[G * N * 3 * 4 + f];
    }
    // h_i
    T hi[DIN];
#pragma unroll
    for (int m = 0; m < DIN; ++m) {
      if constexpr (L == 0) hi[m] = (diag && dir) ? hf[m].d1 : T(0);
      else hi[m] = hb[(i * 49 + lane) * NH + m];
    }
    // convolutional layer c = tanh(mean_4(f w) + b) (network_blocks.py:106-116)
    const T* cn = ly + LC::cn + i * LC::QM * 2;
    T cq[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      T z = T(0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int idx = 4 * q + s;
        T F;
        if (idx < DIN) F = hi[idx];
        else if (idx < 2 * DIN) F = g1[0][idx - DIN];
        else if (idx < 3 * DIN) F = g1[1][idx - 2 * DIN];
        else if (idx < 3 * DIN + 4) F = g2[0][idx - 3 * DIN];
        else F = g2[1][idx - 3 * DIN - 4];
        z += convw[i * DF + idx] * F;
      }
      // the conv's mean_4 factor 1/4 is folded into the LapCache's node weights (adjoint pass)
      cq[q] = cn[2 * q] * z;
      acc += cn[2 * q + 1] * z * z;
    }
    // single linear + tanh + residual (nn.py:296-300)
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      T z = T(0);
#pragma unroll
      for (int q = 0; q < Q; ++q) z += sngw[q * NH + f] * cq[q];
      const T s1 = snv[2 * f] * z;
      acc += snv[2 * f + 1] * z * z;
      hb[(i * 49 + lane) * NH + f] = (DIN == NH) ? (hi[f] + s1) * RSQ2 : s1;
    }
  };
  const cptr<T> Lrow = Lpt;   // record (le, i) at Lrow + i * PS
  Rec c0, c1;
  const int i1 = wv + W < N ? wv + W : wv;
  c0.load(Lrow + wv * PS, P, le, wv);
  c1.load(Lrow + i1 * PS, P, le, i1);
#pragma unroll 1
  for (int i = wv; i < N; i += 2 * W) {
    Rec n0, n1;
    const int i2 = i + 2 * W < N ? i + 2 * W : i, i3 = i + 3 * W < N ? i + 3 * W : i;
    n0.load(Lrow + i2 * PS, P, le, i2);
    n1.load(Lrow + i3 * PS, P, le, i3);
    // fenced, so that the loads stay at the top and the copies into c0, c1 (which wait for them) at the end
    __builtin_amdgcn_sched_barrier(0);
    column(i, c0);
    if (i + W < N) column(i + W, c1);
    __builtin_amdgcn_sched_barrier(0);
    c0 = n0;
    c1 = n1;
  }
}

// E4's determinant term ss = Re sum_{r,s} S_rs S_sr, S_rs = sum_f U_rf Q_f[r,s], on the matrix
// cores.  ss = u^T K u with u = U[(r,f)] (this direction's column of dh/dx of electron
// rowsrc[r], hb) and
//   K[(r,f),(s,g)] = Re(Q_f[r,s] Q_g[s,r])          (4N x 4N, symmetric, the same for every direction),
// so V = K U for all 3N directions at once is one (4N x 4N) x (4N x 48) product:
// v_mfma_{f32,f64}_16x16x4 with K-step s = electron s (k = unit g = lane >> 4), M-tiles over
// rows (r, f), N-tile c = coordinate (column e = lane & 15 of tile c is direction lane 16c + e,
// the hb column).  The A fragment (one K entry per lane) is formed from two LDS reads of Q_f;
// the B fragment is read from hb as it stands.  Then ss = sum_i U[i] V[i] per direction: a
// lane-local sum over the accumulator rows and a sum over the four lane groups.  Multi-wave
// mode: wave wv takes the K-steps s = wv, wv + W, ... (ss is linear in V).  Replaces ~1,650
// VALU FMAs and ~1,100 broadcast LDS reads per wave (the double loop over r < s) by 12 N MFMAs.
// Opt-in (-DAQ_LAP_MFMA_SS): measured SLOWER on N2 / 4096 walkers (local-energy pair 240.8 /
// 241.2 us against 234.0 / 234.6 us with the VALU loop, two interleaved runs, same box;
// profiles/r03_s1_lap_mfma_ab.txt).  The quadratic form does 4x the FLOPs of the S_rs S_sr
// loop (K is 4N x 4N dense, S is rank-structured), and f32 MFMA runs at the f32 VALU rate on
// gfx950, so the matrix cores only pay where they overlap VALU work of the other wave.
template <typename T> struct MfmaTile;
template <> struct MfmaTile<float> {
  typedef float v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // accumulator register v of lane group q holds row 4q + v (column = lane & 15)
  static constexpr __device__ int row(int q, int v) { return 4 * q + v; }
};
template <> struct MfmaTile<double> {
  typedef double v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static constexpr __device__ int row(int q, int v) { return q + 4 * v; }   // f64 C/D map
};

template <typename T, int N>
__device__ __forceinline__ T ss_mfma(const T* Qs, const T* hb, const int* rowsrc, int lane, int wv, int W) {
  static_assert(NH == 4, "K-step = one electron's 4 units");
  using MT = MfmaTile<T>;
  using V4 = typename MT::v4;
  constexpr int NM = (4 * N + 15) / 16;   // M-tiles over the rows (r, f)
  const int q = lane >> 4, e = lane & 15;
  T out = T(0);
  // one N-tile (coordinate c) at a time: 4 NM accumulator registers live instead of 12 NM
#pragma unroll 1
  for (int c = 0; c < 3; ++c) {
    V4 acc[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) acc[m] = V4{T(0), T(0), T(0), T(0)};
#pragma unroll 2
    for (int s = wv; s < N; s += W) {
      const T bop = hb[(rowsrc[s] * 49 + 16 * c + e) * NH + q];
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int i = 16 * m + e;            // A row (r, f); A column k = unit q of electron s
        const int r = i >> 2, f = i & 3;
        const int rc = r < N ? r : N - 1;
        const T* a = Qs + ((rc * N + s) * NH + f) * 2;
        const T* b = Qs + ((s * N + rc) * NH + q) * 2;
        T kv = a[0] * b[0] - a[1] * b[1];
        if (4 * N % 16 != 0 && m == NM - 1) kv = r < N ? kv : T(0);
        acc[m] = MT::mma(kv, bop, acc[m]);
      }
    }
    T p = T(0);
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = 16 * m + MT::row(q, v);
        const int r = i >> 2, f = i & 3;
        if (16 * (m + 1) <= 4 * N || r < N) p += hb[(rowsrc[r < N ? r : N - 1] * 49 + 16 * c + e) * NH + f] * acc[m][v];
      }
    p += __shfl_xor(p, 16);
    p += __shfl_xor(p, 32);
    out = (q == c) ? p : out;
  }
  return out;
}

// One workgroup of W = blockDim.x / 64 waves per walker (W = 1, 2 or 4; aiqmc.hip picks W so
// that small batches still fill the chip): every wave evaluates the per-electron stage of all
// electrons (its lanes are the 3N directions), the h-stream columns i = wv, wv + W, ... of each
// layer and the determinant rows r of its share; per-lane partial sums are combined by wave 0 in
// fixed order.  W = 1 is the single-wave kernel (same arithmetic, same order).
// WMAX: the instantiation's largest W (1: the single-wave kernel, compiled as before for 64
// threads; 4: W = 2 or 4 at run time).
// PH: the phase theta = arg psi instead of log|psi| (complex_output=True, hamiltonian.py:110-130):
// with the LapCache of the PH adjoint pass, every determinant term takes the imaginary part of the
// complex quantity whose real part the log|psi| pass takes (d^2 log det = tr(B d^2A) - tr(B dA B dA)
// is complex; theta = Im log det); the Jastrow factors are real and drop out.  Outputs: el[conf] =
// sum_dir d^2 theta / dx^2 (no potential, no |grad|^2), grad = grad theta.
#ifndef AQ_LAP_WPE
#define AQ_LAP_WPE 2
#endif
template <typename T, int N, int A, int WMAX, bool PH = false>
__global__ __launch_bounds__(64 * WMAX) __attribute__((amdgpu_waves_per_eu(AQ_LAP_WPE))) void k_walker_lap(KArgs ka) {
  using Ly = Lay<N, A>;
  using LC = LapCache<N, A>;
  using SM = SmemLap<T, N, A>;
  constexpr int D0 = 4 * A;
  const cptr<T> P = param_ptr<T>(ka.prm);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* sm = (T*)smem_raw;
  T* xs = sm + SM::xs;
  T* ly = sm + SM::ly;
  T* hb = sm + SM::hb;

  const int conf = xcd_major(blockIdx.x, gridDim.x);   // same walker -> XCD map as the adjoint pass
  const int lane = threadIdx.x & 63;
  const int wv = WMAX == 1 ? 0 : (int)(threadIdx.x >> 6), W = WMAX == 1 ? 1 : (int)(blockDim.x >> 6);
  const bool w0 = wv == 0;
  const int lc = lane >> 4;
  const int er = lane & 15;
  const int le = er < N ? er : N - 1;
  const bool val = (lc == 3);
  const bool live = er < N;
  const bool dir = (lc < 3) && live;
  const int nup = ka.nup;
  const int l49 = lane < 48 ? lane : 48;
  T* yd = sm + SM::yd;
  const cptr<T> Lc = param_ptr<T>((const T*)ka.lapcache + (size_t)conf * LC::size);
  const cptr<T> Lpt = Lc + LC::pt + le * N * LC::pt_n;   // pair records of the lane's row le
  const int rsl = ka.rowsrc[lane < N ? lane : N - 1];      // determinant row lane's electron (E3, E4)
  const int rsle = ka.rowsrc[le];                          // and row le's (E2)
#ifdef AQ_PHASE_PROF
  unsigned long long t_ph = __builtin_readcyclecounter();
#endif

  if (w0 && lane < 3 * N) xs[lane] = ((const T*)ka.pos)[(size_t)conf * 3 * N + lane];
  T h0b[D0];
#pragma unroll
  for (int m = 0; m < D0; ++m) h0b[m] = Lc[LC::h0b + le * D0 + m];
  static_assert(LC::layer_n * sizeof(T) % 16 == 0 && SM::ly * sizeof(T) % 16 == 0, "16-byte staging");
  stage_copy<T>(ly, Lc, LC::layer_n);
  __syncthreads();

  // ------------------------------------------------------------------ per-electron stage (electron.h)
  ElecOut<T, A> eo;
  electron_stage<T, N, A>(P, xs + le * 3, le, lc, eo);
  T vv = (!PH && w0 && val && live) ? eo.ven : T(0);
  T acc = T(0);   // curvature sources, per direction lane
#pragma unroll
  for (int m = 0; m < D0; ++m) acc += h0b[m] * eo.hf[m].d2;   // ae features as leaves
  if (!w0) acc = T(0);
  // Yt row of electron le, first and second derivatives (nn.py:449-452, 479-485) -> LDS
#pragma unroll
  for (int col = 0; col < N; ++col) {
    PJ<T> s = P[Ly::wy + col] * eo.yst[0];
#pragma unroll
    for (int m = 1; m < NYW; ++m) s = s + P[Ly::wy + m * N + col] * eo.yst[m];
    const PJ<T> yt = eo.env * s;
    if (w0) {
      yd[col * 49 + l49] = yt.d1;
      yd[(N + col) * 49 + l49] = yt.d2;
    }
  }
  LPH(0);
  T jd1 = (!PH && w0 && dir) ? eo.jae.d1 : T(0);
  T jd2 = (!PH && w0 && dir) ? eo.jae.d2 : T(0);

  // ------------------------------------------------------------------ h stream, first derivatives
  // kLapPrefetch: each staged block's loads are issued one phase ahead (into spare VGPRs: the kernel
  // runs at 2 waves/SIMD, 256 VGPRs each) and written to LDS after the barrier that frees it, so
  // no wave waits a whole L2/HBM round trip at a stage boundary
  LPH(1);
  StageRegs<T, LC::layer_n> lnext;
  if constexpr (kLapPrefetch) lnext.load(Lc + LC::layer_n);
  lap_layer<T, N, A, 0>(P, xs, hb, ly, eo.hf, l49, lc, er, le, val, dir, live, nup, jd1, jd2, vv, acc, wv, W, Lpt);
  LPH(2);
  if constexpr (PH) {   // the e-e Jastrow terms and V_ee of layer 0's column loop: not part of theta
    jd1 = jd2 = vv = T(0);
  }
  __syncthreads();
  if constexpr (kLapPrefetch) lnext.store(ly);
  else stage_copy<T>(ly, Lc + LC::layer_n, LC::layer_n);
  __syncthreads();
  if constexpr (kLapPrefetch) lnext.load(Lc + 2 * LC::layer_n);
  lap_layer<T, N, A, 1>(P, xs, hb, ly, eo.hf, l49, lc, er, le, val, dir, live, nup, jd1, jd2, vv, acc, wv, W, Lpt);
  __syncthreads();
  if constexpr (kLapPrefetch) lnext.store(ly);
  else stage_copy<T>(ly, Lc + 2 * LC::layer_n, LC::layer_n);
  __syncthreads();
  LPH(3);
  StageRegs<T, 8 * N * N> qnext;
  StageRegs<T, (SM::stage_b ? 2 * N * N : 4)> bnext;
  if constexpr (kLapPrefetch) {
    qnext.load(Lc + LC::qs);
    if constexpr (SM::stage_b) bnext.load(Lc + LC::bm);
  }
  // E2's Phi row of electron le, issued a layer ahead (per-lane 16-byte loads of 2N contiguous values)
  T phrow[2 * N];
  if constexpr (2 * N % 4 == 0) ld_vec<T, 2 * N>(Lc + LC::ph + le * N * 2, phrow);
  else {
#pragma unroll
    for (int k = 0; k < 2 * N; ++k) phrow[k] = Lc[LC::ph + le * N * 2 + k];
  }
  lap_layer<T, N, A, 2>(P, xs, hb, ly, eo.hf, l49, lc, er, le, val, dir, live, nup, jd1, jd2, vv, acc, wv, W, Lpt);
  if (W > 1) __syncthreads();   // the determinant terms read every wave's columns of dh/dx

  LPH(4);
  // ------------------------------------------------------------------ determinant terms
  // (phases fenced so that the scheduler does not stretch their live ranges across each other)
  const int* rowsrc = ka.rowsrc;
  const T* Qs = nullptr;                     // LDS copy, set after E1
  const T* Bu = (const T*)(Lc + LC::bm);     // LDS copy after E1 where it fits
  const cptr<T> Ph = Lc + LC::ph;
  // row r's electron rowsrc[r] by a lane read of rsl (lane r holds it, loaded at kernel start): read
  // through the pointer, every (r, s) step of E3/E4 was a dependent global load (the kernel also writes
  // global memory, so it cannot be a scalar load) waited for before its LDS address was known
#define UH(r, f) hb[(__builtin_amdgcn_readlane(rsl, (r)) * 49 + l49) * NH + (f)]
  // E1: Yt row jets of electron le (stored after the per-electron stage)
  T Yd1[N], Yd2[N];
#pragma unroll
  for (int col = 0; col < N; ++col) {
    Yd1[col] = yd[col * 49 + l49];
    Yd2[col] = yd[(N + col) * 49 + l49];
  }
  __builtin_amdgcn_sched_barrier(0);
  // Q_f (and B) to LDS over the dead layer block and Yt jets: E2-E4 read them at wave-uniform
  // and per-lane offsets; their scalar loads from L2 were E4's latency chain
  __syncthreads();   // every wave has read its Yt jets (E1)
  {
    T* qd = sm + SM::qs;
    static_assert(LC::qs % 4 == 0 && LC::bm % 4 == 0 && SM::qs % 4 == 0 && SM::bs % 4 == 0, "16-byte staging");
    if constexpr (kLapPrefetch) {
      qnext.store(qd);
      if constexpr (SM::stage_b) bnext.store(sm + SM::bs);
    } else {
      stage_copy<T>(qd, Lc + LC::qs, 8 * N * N);
      if constexpr (SM::stage_b) {
        T* bd = sm + SM::bs;
        stage_copy<T>(bd, Lc + LC::bm, 2 * N * N);
      }
    }
  }
  __syncthreads();
  Qs = sm + SM::qs;
  if constexpr (SM::stage_b) Bu = sm + SM::bs;
  LPH(5);
  // E2: w = Phi[e,:] * dYt[e,:], w.b_e, and t2 = Re sum_col (2 dPhi[e,col] Yt'[col] +
  //     Phi[e,col] Yt''[col]) B[col,e] with e = le (U of row e)
  const int spe = le < nup ? 0 : 1;
  T Ue[NH];
#pragma unroll
  for (int f = 0; f < NH; ++f) Ue[f] = hb[(rsle * 49 + l49) * NH + f];   // U of row le (per lane)
  T wr[N], wi[N];
  T wbr = T(0), wbi = T(0), t2 = T(0);
#pragma unroll
  for (int col = 0; col < N; ++col) {
    const T pr = phrow[2 * col], pm = phrow[2 * col + 1];
    const T br = Bu[(col * N + le) * 2], bi = Bu[(col * N + le) * 2 + 1];
    wr[col] = pr * Yd1[col];
    wi[col] = pm * Yd1[col];
    wbr += wr[col] * br - wi[col] * bi;
    wbi += wr[col] * bi + wi[col] * br;
    // d Phi[e, col] / dx for both spin blocks from wave-uniform weights (scalar loads, re-read per
    // column through an opaque pointer), selected by the row's spin: the per-lane weight loads
    // (spin-dependent address) were hoisted into registers and spilled
    cptr<T> Pw = P;
    asm volatile("" : "+s"(Pw));
    T d0r = T(0), d0i = T(0), d1r = T(0), d1i = T(0);
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      d0r += Ue[f] * Pw[Ly::orb_w + (f * N + col) * 2];
      d0i += Ue[f] * Pw[Ly::orb_w + (f * N + col) * 2 + 1];
      d1r += Ue[f] * Pw[Ly::orb_w + ((NH + f) * N + col) * 2];
      d1i += Ue[f] * Pw[Ly::orb_w + ((NH + f) * N + col) * 2 + 1];
    }
    const T dpr = spe ? d1r : d0r, dpi = spe ? d1i : d0i;
    const T xr = T(2) * dpr * Yd1[col] + pr * Yd2[col];
    const T xi = T(2) * dpi * Yd1[col] + pm * Yd2[col];
    t2 += PH ? xr * bi + xi * br : xr * br - xi * bi;
  }
  // t2 is consumed only at the end of the kernel: left alone, the compiler sinks E2's dPhi arithmetic
  // past E4 while its weight loads stay here, and spills the weights (a scalar load, wait and lane
  // write per weight pair; 193 VGPRs, 159 SGPRs spilled).  Pinned here (with the Phi row prefetched a
  // layer ahead, above): 187 VGPRs, 34 spilled SGPRs.  Measured (N2, interleaved): pinned alone, the
  // multi-wave instantiation gains 4-5 % and the one-wave one loses 4.5 % (E2's Phi loads then sit on
  // its path; profiles/r06_s9_ab_lap_e2pin.txt); pinned with the Phi row prefetch, the one-wave
  // instantiation gains 2 % (E_L pair 169.8-171.0 -> 166.6-167.3 us at 4,096 walkers, fp64 bitwise,
  // profiles/r06_s9_ab_lap_e2ph.txt)
  asm volatile("" : "+v"(t2));
  __builtin_amdgcn_sched_barrier(0);
  LPH(6);
  // E3: gradient: sum_{r,f} U Re Q_f[r,r] + Re(w . b_e) + Jastrow  (rows r = wv, wv + W, ...)
  T g = w0 ? jd1 + (PH ? wbi : wbr) : jd1;
#pragma unroll 2
  for (int r = wv; r < N; r += W)
#pragma unroll
    for (int f = 0; f < NH; ++f) g += UH(r, f) * Qs[((r * N + r) * NH + f) * 2 + (PH ? 1 : 0)];
  LPH(7);
  // E4: cross = Re sum_r z_r S_re (z = B^T w);  ss = Re sum_{r,s} S_rs S_sr,  S_rs = sum_f U_rf Q_f[r,s]
  // (row r costs N - r: wave wv takes rows wv, 2W-1-wv, 2W+wv, ... so the shares balance)
  T cross = T(0), ss = T(0);
#ifndef AQ_LAP_E4R_UNROLL
#define AQ_LAP_E4R_UNROLL 1
#endif
#pragma unroll AQ_LAP_E4R_UNROLL
  for (int t = 0; t * W < N; ++t) {
    const int r = t * W + ((t & 1) ? W - 1 - wv : wv);
    if (r >= N) continue;
    T ur[NH];
#pragma unroll
    for (int f = 0; f < NH; ++f) ur[f] = UH(r, f);
    T zr = T(0), zi = T(0);
#pragma unroll
    for (int col = 0; col < N; ++col) {
      const T br = Bu[(col * N + r) * 2], bi = Bu[(col * N + r) * 2 + 1];
      zr += br * wr[col] - bi * wi[col];
      zi += br * wi[col] + bi * wr[col];
    }
    T sr = T(0), si = T(0);
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      sr += ur[f] * Qs[((r * N + le) * NH + f) * 2];
      si += ur[f] * Qs[((r * N + le) * NH + f) * 2 + 1];
    }
    cross += PH ? zr * si + zi * sr : zr * sr - zi * si;
#ifndef AQ_LAP_MFMA_SS
    constexpr bool vss = true;
#else
    constexpr bool vss = PH;   // the MFMA form of ss is built for the real part only
#endif
    if constexpr (vss) {
    T dr = T(0), di = T(0);
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      dr += ur[f] * Qs[((r * N + r) * NH + f) * 2];
      di += ur[f] * Qs[((r * N + r) * NH + f) * 2 + 1];
    }
    ss += PH ? T(2) * dr * di : dr * dr - di * di;
#ifndef AQ_LAP_E4_UNROLL
#define AQ_LAP_E4_UNROLL 1
#endif
#pragma unroll AQ_LAP_E4_UNROLL
    for (int s = r + 1; s < N; ++s) {
      T ar = T(0), ai = T(0), br = T(0), bi = T(0);
#pragma unroll
      for (int f = 0; f < NH; ++f) {
        const T us = UH(s, f);
        ar += ur[f] * Qs[((r * N + s) * NH + f) * 2];
        ai += ur[f] * Qs[((r * N + s) * NH + f) * 2 + 1];
        br += us * Qs[((s * N + r) * NH + f) * 2];
        bi += us * Qs[((s * N + r) * NH + f) * 2 + 1];
      }
      ss += T(2) * (PH ? ar * bi + ai * br : ar * br - ai * bi);
    }
    }
  }
#ifdef AQ_LAP_MFMA_SS
  if constexpr (!PH) {
    __builtin_amdgcn_sched_barrier(0);
    ss = ss_mfma<T, N>(Qs, hb, rowsrc, lane, wv, W);
  }
#endif
#undef UH
  LPH(8);
  // (w.b_e)^2: its real part, or (PH) its imaginary part 2 Re Im
  const T wb2 = PH ? T(2) * wbr * wbi : wbr * wbr - wbi * wbi;
  T lap = (w0 ? t2 : T(0)) - (ss + T(2) * cross + (w0 ? wb2 : T(0))) + jd2 + acc;
  if (W > 1) {
    // partial sums of waves 1..W-1 -> wave 0, added in wave order (the ly block is free now)
    __syncthreads();
    if (!w0) {
      T* red = ly + (wv - 1) * 3 * 64;   // spans ly, hb, yd: all read for the last time above
      red[lane] = g;
      red[64 + lane] = lap;
      red[128 + lane] = vv;
    }
    __syncthreads();
    if (!w0) return;
    for (int k = 1; k < W; ++k) {
      const T* red = ly + (k - 1) * 3 * 64;
      g += red[lane];
      lap += red[64 + lane];
      vv += red[128 + lane];
    }
  }

  LPH(9);
  // ------------------------------------------------------------------ outputs
  const T gd = dir ? g : T(0);
  if constexpr (PH) {
    // the phase Laplacian sum_dir d^2 theta / dx^2 (incl. the adjoint pass's pair-local part) and grad theta
    const T lsum = wave_sum(dir ? lap : T(0)) + Lc[LC::scal];
    if (ka.grad && dir) ((T*)ka.grad)[(size_t)conf * 3 * N + 3 * le + lc] = g;
    if (lane == 0 && ka.el) ((T*)ka.el)[conf] = lsum;
    return;
  }
  const T sumsq = wave_sum(gd * gd);
  if (ka.grad && dir) ((T*)ka.grad)[(size_t)conf * 3 * N + 3 * le + lc] = g;
  const T kin = T(-0.5) * (wave_sum(dir ? lap : T(0)) + Lc[LC::scal] + sumsq);   // hamiltonian.py:126-127
  const T pot = wave_sum(vv) + P[Ly::vnn];
  if (lane == 0) {
    if (ka.el) ((T*)ka.el)[conf] = pot + kin;
    if (ka.sumsq) ((T*)ka.sumsq)[conf] = sumsq;
  }
}

}  // namespace aq
