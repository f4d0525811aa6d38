// walker_pgrad.h -- per-walker parameter gradient O_b = d log|psi(x_b)| / d theta of the
// AIQMC network (the psi_tangent of the energy-gradient custom JVP,
// Loss/loss.py:242-265, and of the Adam step, Optimizer/adam.py:49-59).
//
// One wave per PgK walkers (four for N <= 4, two for N <= 8, one above); not on the Metropolis hot
// path (one launch per optimisation step), so the kernel favours clarity: a plain forward pass
// with every intermediate kept in LDS (lanes over items: electrons, pairs, (electron, unit),
// (row, column) of every walker of the wave), Gauss-Jordan of gj.h per walker, then the reverse
// pass with the parameter adjoints accumulated in an LDS copy of the kernel parameter layout
// (Lay<N,A>) per walker by LDS atomics and written out per walker.
//
// Adjoints (L = log|det A| + J_ee + J_ae, Q11; B = A^{-1}, A = Phi (.) Yt):
//   dL/dPhi_re[r,c] = Re B[c,r] Yt[r,c],  dL/dPhi_im[r,c] = -Im B[c,r] Yt[r,c],
//   dL/dYt[r,c] = Re(B[c,r] Phi[r,c]);  Phi[r,:] = H[src r,:] W_s + b_s  (nn.py:432-456);
//   Yt[r,c] = env_r sum_m y[r,m] What[m,c]  (What = row-normalised W_y, nn.py:449-452: the
//   normalisation is undone on the canonical side, aiqmc_logpsi_param_grad);
//   h stream (nn.py:280-311, network_blocks.py:106-116), pair stream (nn.py:305-309),
//   Ynlm stream (nn.py:313-341), envelope (envelope.py:26-30), Pade Jastrows (Jastrow.py).
#pragma once
#include "electron.h"
#include "gj.h"
#include "jets.h"
#include "layout.h"
#include "walker_kernel.h"

namespace aq {

template <typename T, int N, int A>
struct SmemPG {
  static constexpr int D0 = 4 * A;
  static constexpr int DFM = 3 * D0 + 2 * NH2;
  static constexpr int QM = DFM / 4;
  static constexpr int xs = 0;                            // [48]
  static constexpr int pg = 48;                           // [Lay::total] d L / d (kernel parameter)
  static constexpr int hl = pg + Lay<N, A>::total;        // [4][N][D0] h^0..h^3 (h^l width D0 for l = 0, 4 after)
  static constexpr int g1 = hl + 4 * N * D0;              // [3][2][D0] group means of h^l
  static constexpr int g2 = g1 + 6 * D0;                  // [3][2][N][4] column means of h2^(l)
  static constexpr int cq = g2 + 24 * N;                  // [3][N][QM] conv outputs
  static constexpr int sv = cq + 3 * N * QM;              // [3][N][4] single outputs
  static constexpr int env = sv + 12 * N;                 // [N] envelope of row r
  static constexpr int yst = env + N;                     // [N][6] Ynlm stream output
  static constexpr int yv = yst + NYW * N;                // [N][N] Yt
  static constexpr int ph = yv + N * N;                   // [N][N][2] Phi
  static constexpr int mx = ph + 2 * N * N;               // [N][N][2] B = A^{-1}
  static constexpr int hb = mx + 2 * N * N;               // [N][4] adjoint of h^{l+1}
  static constexpr int hn = hb + 4 * N;                   // [N][4] adjoint of h^l
  static constexpr int g2b = hn + 4 * N;                  // [3][2][N][4] adjoints of g2
  static constexpr int ybar = g2b + 24 * N;               // [N][N] adjoint of Yt
  static constexpr int fb = ybar + N * N;                 // [N][DFM] adjoints of the conv inputs
  static constexpr int zc = fb + N * DFM;                 // [N][QM] conv pre-activation adjoints
  static constexpr int zs = zc + N * QM;                  // [N][4]  single pre-activation adjoints
  static constexpr int red = zs + 4 * N;                  // [2] J sums
  static constexpr int end = red + 2;
  static constexpr int bytes = ((end * (int)sizeof(T)) + 15) & ~15;
  static constexpr int hoff(int l) { return l * N * D0; }
};

template <typename T> __device__ __forceinline__ void lds_add(T* p, T v) { atomicAdd(p, v); }

// Walkers per wave: every phase below is a loop of lanes over items (electrons, pairs, (electron,
// unit), (row, column), parameters), which for a small system leaves most lanes idle (N = 4: 16
// pairs, 16 (electron, unit) items, 4 electrons); PGK walkers share a wave by widening each loop to
// PGK x items (walker k = item / n), each walker with its own LDS block.  The Gauss-Jordan (gj.h,
// one matrix per wave) runs once per walker.  Per walker the arithmetic and its order are those of
// the one-walker kernel (PGK = 1).
#ifndef AQ_PGK1
template <int N> struct PgK { static constexpr int value = N <= 4 ? 4 : (N <= 8 ? 2 : 1); };
#else   // A/B builds: one walker per wave
template <int N> struct PgK { static constexpr int value = 1; };
#endif

template <typename T, int N, int A, int K = 1>
__global__ __launch_bounds__(64) void k_param_grad(KArgs ka) {
  using Ly = Lay<N, A>;
  using SM = SmemPG<T, N, A>;
  constexpr int D0 = SM::D0;
  constexpr int QM = SM::QM;
  constexpr int ST = SM::bytes / (int)sizeof(T);   // one walker's LDS block (16-byte multiple)
  const cptr<T> P = param_ptr<T>(ka.prm);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* const sm0 = (T*)smem_raw;
  const int lane = threadIdx.x;
  const int nup = ka.nup;
  const T gw[2] = {T(1) / T(nup), T(1) / T(N - nup)};
  const T RSQ2 = T(0.70710678118654752);
  const int* rowsrc = ka.rowsrc;
  const int conf0 = blockIdx.x * K;
  const int nk = ka.nconf - conf0 < K ? ka.nconf - conf0 : K;   // walkers of this wave
  // walker k's LDS block (and its pieces)
  auto S = [&](int k) { return sm0 + k * ST; };

  for (int it = lane; it < nk * 3 * N; it += 64) {
    const int k = it / (3 * N), j = it - k * 3 * N;
    S(k)[SM::xs + j] = ((const T*)ka.pos)[(size_t)(conf0 + k) * 3 * N + j];
  }
  for (int it = lane; it < K * Ly::total; it += 64) {
    const int k = it / Ly::total;
    S(k)[SM::pg + it - k * Ly::total] = T(0);
  }
  for (int it = lane; it < K * 24 * N; it += 64) {
    const int k = it / (24 * N);
    S(k)[SM::g2 + it - k * 24 * N] = T(0);
  }
  if (lane < 2 * K) S(lane >> 1)[SM::red + (lane & 1)] = T(0);
  __syncthreads();

  // ---------------------------------------------------------------- forward: electron stage
  if (lane < nk * N) {
    const int k = lane / N, i = lane - k * N;
    T* sm = S(k);
    ElecOut<T, A> eo;
    electron_stage<T, N, A>(P, sm + SM::xs + 3 * i, i, 3, eo);
#pragma unroll
    for (int m = 0; m < D0; ++m) sm[SM::hl + i * D0 + m] = eo.hf[m].v;
#pragma unroll
    for (int m = 0; m < NYW; ++m) sm[SM::yst + i * NYW + m] = eo.yst[m].v;
    sm[SM::env + i] = eo.env.v;
    for (int c = 0; c < N; ++c) {
      T y = T(0);
#pragma unroll
      for (int m = 0; m < NYW; ++m) y += eo.yst[m].v * P[Ly::wy + m * N + c];
      sm[SM::yv + i * N + c] = eo.env.v * y;
    }
    lds_add(&sm[SM::red], eo.jae.v);
  }
  // ---------------------------------------------------------------- forward: pair stream column means
  for (int it = lane; it < nk * N * N; it += 64) {
    const int kw = it / (N * N), idx = it - kw * N * N;
    T* sm = S(kw);
    const T* xs = sm + SM::xs;
    const int k = idx / N, i = idx - k * N;
    const bool diag = k == i;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = xs[3 * i + c] - xs[3 * k + c];
    const T r = f_sqrt(diag ? T(1) : d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    T p[4] = {diag ? T(0) : r, diag ? T(0) : d[0], diag ? T(0) : d[1], diag ? T(0) : d[2]};
    if (k < i) lds_add(&sm[SM::red + 1], f_div(P[Ly::jee_c + k * N + i] * r, P[Ly::jee_a + k * N + i] * r + T(1)));
    const int G = k >= nup ? 1 : 0;
#pragma unroll
    for (int f = 0; f < 4; ++f) lds_add(&sm[SM::g2 + ((0 * 2 + G) * N + i) * 4 + f], p[f] * gw[G]);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const cptr<T> dw = P + (j == 0 ? Ly::dbl_w0 : Ly::dbl_w1);
      const cptr<T> db = P + (j == 0 ? Ly::dbl_b0 : Ly::dbl_b1);
      T q[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        T s = db[o];
#pragma unroll
        for (int m = 0; m < 4; ++m) s += p[m] * dw[m * 4 + o];
        q[o] = f_tanh(s);
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        p[o] = (p[o] + q[o]) * RSQ2;
        lds_add(&sm[SM::g2 + (((j + 1) * 2 + G) * N + i) * 4 + o], p[o] * gw[G]);
      }
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- forward: h stream (nn.py:280-311)
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const int d = l == 0 ? D0 : NH;
    const int DF = 3 * d + 2 * NH2, Q = DF / 4;
    for (int it = lane; it < nk * 2 * d; it += 64) {   // 2 K D0 > 64 lanes for A >= 3
      const int kw = it / (2 * d), gl = it - kw * 2 * d;
      T* sm = S(kw);
      const T* h = sm + SM::hl + SM::hoff(l);
      T* g1 = sm + SM::g1 + l * 2 * D0;
      const int G = gl / d, m = gl - G * d;
      T s = T(0);
      for (int k = (G ? nup : 0); k < (G ? N : nup); ++k) s += h[k * d + m];
      g1[G * D0 + m] = s * gw[G];
    }
    __syncthreads();
    const cptr<T> convw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2));
    const cptr<T> convb = P + (l == 0 ? Ly::conv_b0 : (l == 1 ? Ly::conv_b1 : Ly::conv_b2));
    for (int it = lane; it < nk * N * Q; it += 64) {
      const int kw = it / (N * Q), idx = it - kw * N * Q;
      T* sm = S(kw);
      const T* h = sm + SM::hl + SM::hoff(l);
      const T* g1 = sm + SM::g1 + l * 2 * D0;
      const int i = idx / Q, q = idx - i * Q;
      T z = T(0);
      for (int s4 = 0; s4 < 4; ++s4) {
        const int j = 4 * q + s4;
        T F;
        if (j < d) F = h[i * d + j];
        else if (j < 3 * d) F = g1[((j - d) / d) * D0 + (j - d) % d];
        else F = sm[SM::g2 + ((l * 2 + (j - 3 * d) / 4) * N + i) * 4 + ((j - 3 * d) & 3)];
        z += F * convw[i * DF + j];
      }
      sm[SM::cq + (l * N + i) * QM + q] = f_tanh(z * T(0.25) + convb[i * Q + q]);
    }
    __syncthreads();
    const cptr<T> sngw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
    const cptr<T> sngb = P + (l == 0 ? Ly::sng_b0 : (l == 1 ? Ly::sng_b1 : Ly::sng_b2));
    for (int it = lane; it < nk * N * NH; it += 64) {
      const int kw = it / (N * NH), idx = it - kw * N * NH;
      T* sm = S(kw);
      const T* h = sm + SM::hl + SM::hoff(l);
      const int i = idx / NH, f = idx - i * NH;
      T z = sngb[f];
      for (int q = 0; q < Q; ++q) z += sm[SM::cq + (l * N + i) * QM + q] * sngw[q * NH + f];
      const T s = f_tanh(z);
      sm[SM::sv + (l * N + i) * NH + f] = s;
      sm[SM::hl + SM::hoff(l + 1) + i * NH + f] = (d == NH) ? (h[i * d + f] + s) * RSQ2 : s;
    }
    __syncthreads();
  }
  // ---------------------------------------------------------------- forward: Phi, Gauss-Jordan (nn.py:432-506)
  for (int it = lane; it < nk * N * N; it += 64) {
    const int kw = it / (N * N), idx = it - kw * N * N;
    T* sm = S(kw);
    const T* H3 = sm + SM::hl + SM::hoff(3);
    const int r = idx / N, c = idx - r * N;
    const int src = rowsrc[r], s = r < nup ? 0 : 1;
    T re = P[Ly::orb_b + (s * N + c) * 2], im = P[Ly::orb_b + (s * N + c) * 2 + 1];
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      re += H3[src * NH + f] * P[Ly::orb_w + ((s * NH + f) * N + c) * 2];
      im += H3[src * NH + f] * P[Ly::orb_w + ((s * NH + f) * N + c) * 2 + 1];
    }
    sm[SM::ph + idx * 2] = re;
    sm[SM::ph + idx * 2 + 1] = im;
  }
  __syncthreads();
  T logdet[K], phr[K], phi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k < nk) {
      T* sm = S(k);
      gj_inverse<T, N>(sm + SM::ph, sm + SM::yv, sm + SM::mx, lane, logdet[k], phr[k], phi[k]);
    } else {
      logdet[k] = phr[k] = phi[k] = T(0);
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- reverse: orbitals (B1)
  const bool phg = ka.phase_grad != 0;
  for (int it = lane; it < nk * N * N; it += 64) {
    const int kw = it / (N * N), idx = it - kw * N * N;
    T* sm = S(kw);
    T* pg = sm + SM::pg;
    const T* Ph = sm + SM::ph;
    const T* Mx = sm + SM::mx;
    const T* H3 = sm + SM::hl + SM::hoff(3);
    const int r = idx / N, c = idx - r * N;
    const int src = rowsrc[r], s = r < nup ? 0 : 1;
    const T br = Mx[(c * N + r) * 2], bi = Mx[(c * N + r) * 2 + 1];
    const T yt = sm[SM::yv + idx];
    // log|det| = Re ln det: (Re B yt, -Im B yt), dYt = Re(B Phi); phase = Im ln det:
    // (Im B yt, Re B yt), dYt = Im(B Phi)
    const T pr_ = phg ? bi * yt : br * yt, pi_ = phg ? br * yt : -bi * yt;   // dL/dPhi_re, dL/dPhi_im
    sm[SM::ybar + idx] = phg ? br * Ph[idx * 2 + 1] + bi * Ph[idx * 2] : br * Ph[idx * 2] - bi * Ph[idx * 2 + 1];
    lds_add(&pg[Ly::orb_b + (s * N + c) * 2], pr_);
    lds_add(&pg[Ly::orb_b + (s * N + c) * 2 + 1], pi_);
#pragma unroll
    for (int f = 0; f < NH; ++f) {
      lds_add(&pg[Ly::orb_w + ((s * NH + f) * N + c) * 2], H3[src * NH + f] * pr_);
      lds_add(&pg[Ly::orb_w + ((s * NH + f) * N + c) * 2 + 1], H3[src * NH + f] * pi_);
    }
  }
  for (int it = lane; it < nk * N * NH; it += 64) {
    const int kw = it / (N * NH), idx = it - kw * N * NH;
    T* sm = S(kw);
    const T* Mx = sm + SM::mx;
    const int r = idx / NH, f = idx - r * NH;
    const int s = r < nup ? 0 : 1;
    T a = T(0);
    for (int c = 0; c < N; ++c) {
      const T br = Mx[(c * N + r) * 2], bi = Mx[(c * N + r) * 2 + 1];
      const T yt = sm[SM::yv + r * N + c];
      const T wr = P[Ly::orb_w + ((s * NH + f) * N + c) * 2], wi = P[Ly::orb_w + ((s * NH + f) * N + c) * 2 + 1];
      a += phg ? wr * bi * yt + wi * br * yt : wr * br * yt - wi * bi * yt;
    }
    sm[SM::hb + rowsrc[r] * NH + f] = a;
  }
  __syncthreads();
  // ---------------------------------------------------------------- reverse: per electron (Yt row, envelope,
  // e-n Jastrow, Ynlm stream), one lane per (walker, electron)
  if (lane < nk * N) {
    const int kw = lane / N, i = lane - kw * N;
    T* sm = S(kw);
    T* pg = sm + SM::pg;
    const T* xs = sm + SM::xs;
    const T env = sm[SM::env + i];
    T ystb[NYW];
    T envb = T(0);
#pragma unroll
    for (int m = 0; m < NYW; ++m) ystb[m] = T(0);
    for (int c = 0; c < N; ++c) {
      const T yb = sm[SM::ybar + i * N + c];
      T y = T(0);
#pragma unroll
      for (int m = 0; m < NYW; ++m) {
        const T w = P[Ly::wy + m * N + c];
        y += sm[SM::yst + i * NYW + m] * w;
        ystb[m] += env * w * yb;
        lds_add(&pg[Ly::wy + m * N + c], env * sm[SM::yst + i * NYW + m] * yb);
      }
      envb += yb * y;
    }
    // geometry of electron i
    T ae[A][3], ra[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
#pragma unroll
      for (int c = 0; c < 3; ++c) ae[a][c] = xs[3 * i + c] - P[Ly::atoms + a * 3 + c];
      ra[a] = f_sqrt(ae[a][0] * ae[a][0] + ae[a][1] * ae[a][1] + ae[a][2] * ae[a][2]);
    }
    // envelope.py:26-30: env = alpha sum_a e^{-beta r^2} + xi sum_{a,d} sigma e^{-pi ae}
    const T alpha = P[Ly::env_alpha + i], xi = P[Ly::env_xi + i];
    T da = T(0), dxi = T(0);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const T beta = P[Ly::env_beta + i * A + a];
      const T e = f_exp(-beta * ra[a] * ra[a]);
      da += e;
      pg[Ly::env_beta + i * A + a] += envb * (-alpha * ra[a] * ra[a] * e);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const T pi_ = P[Ly::env_pi + (i * A + a) * 3 + c], sg = P[Ly::env_sigma + (i * A + a) * 3 + c];
        const T e2 = f_exp(-pi_ * ae[a][c]);
        dxi += sg * e2;
        pg[Ly::env_sigma + (i * A + a) * 3 + c] += envb * xi * e2;
        pg[Ly::env_pi + (i * A + a) * 3 + c] += envb * (-xi * sg * ae[a][c] * e2);
      }
      // Jastrow.py:84-93: ja = -c34 / (2 beta) (1 - e^{-c14 beta r})
      const T bj = P[Ly::jae_b + i * A + a];
      const T c34 = P[Ly::c34 + a], c14 = P[Ly::c14 + a];
      const T ex = f_exp(-c14 * bj * ra[a]);
      if (!phg)   // the Jastrows are real: no phase
        pg[Ly::jae_b + i * A + a] += c34 / (T(2) * bj * bj) * (T(1) - ex) - c34 / (T(2) * bj) * (c14 * ra[a] * ex);
    }
    pg[Ly::env_alpha + i] += envb * da;
    pg[Ly::env_xi + i] += envb * dxi;
    // Ynlm stream: recompute the three layers of electron i, then reverse (nn.py:313-341)
    constexpr int DY0 = Ly::DY0;
    T y0[DY0];
    {
      // input features (nn.py:156-193, the electron stage's formulas, values only)
      const T PI = T(3.141592653589793);
      const T c0 = T(0.5) * f_sqrt(T(1) / PI), c1 = f_sqrt(T(3) / (T(4) * PI));
      const T k15h = T(0.5) * f_sqrt(T(15) / PI), k5q = T(0.25) * f_sqrt(T(5) / PI);
      const T k15q = T(0.25) * f_sqrt(T(15) / PI), k35 = T(0.25) * f_sqrt(T(35) / (T(2) * PI));
      const T k105h = T(0.5) * f_sqrt(T(105) / PI), k21 = T(0.25) * f_sqrt(T(21) / (T(2) * PI));
      const T k7 = T(0.25) * f_sqrt(T(7) / PI), k105q = T(0.25) * f_sqrt(T(105) / PI);
      T hisum = T(0), spsum = T(0);
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const T rinv = T(1) / ra[a];
        const T x0 = ae[a][0] * rinv, x1 = ae[a][1] * rinv, x2 = ae[a][2] * rinv;
        y0[4 * a] = c0;
        y0[4 * a + 1] = c1 * x0;
        y0[4 * a + 2] = c1 * x1;
        y0[4 * a + 3] = c1 * x2;
        spsum += c0 + c1 * x0 + c1 * x1 + c1 * x2;
        const T y2 = ra[a] * ra[a], inv2 = rinv * rinv, inv3 = inv2 * rinv;
        const T x00 = x0 * x0, x11 = x1 * x1, x22 = x2 * x2, x01 = x0 * x1;
        const T s2 = k15h * x01 + k15h * (x1 * x2) + k5q * (T(3) * x22 - y2) + k15h * (x0 * x2) + k15q * (x00 - x11);
        const T f5 = T(5) * x22 - y2;
        const T s3 = k35 * (x1 * (T(3) * x00 - x11)) + k105h * (x01 * x2) + k21 * (x1 * f5) +
                     k7 * (x2 * (T(5) * x22 - T(3) * y2)) + k21 * (x0 * f5) + k105q * ((x00 - x11) * x2) +
                     k35 * (x0 * (x00 - T(3) * x11));
        hisum += s2 * inv2 + s3 * inv3;
      }
      y0[4 * A] = hisum * (T(1) / T(12 * A));
      y0[4 * A + 1] = spsum * (T(1) / T(4 * A));
    }
    T t0[NYW], y1[NYW], t1[NYW], y2[NYW], t2[NYW];
#pragma unroll
    for (int q = 0; q < NYW; ++q) {
      T s = P[Ly::y_b0 + q];
#pragma unroll
      for (int m = 0; m < DY0; ++m) s += P[Ly::y_w0 + m * NYW + q] * y0[m];
      t0[q] = f_tanh(s);
      y1[q] = (DY0 == NYW) ? RSQ2 * (y0[q < DY0 ? q : 0] + t0[q]) : t0[q];
    }
#pragma unroll
    for (int q = 0; q < NYW; ++q) {
      T s = P[Ly::y_b1 + q];
#pragma unroll
      for (int m = 0; m < NYW; ++m) s += P[Ly::y_w1 + m * NYW + q] * y1[m];
      t1[q] = f_tanh(s);
    }
#pragma unroll
    for (int q = 0; q < NYW; ++q) y2[q] = RSQ2 * (y1[q] + t1[q]);
#pragma unroll
    for (int q = 0; q < NYW; ++q) {
      T s = P[Ly::y_b2 + q];
#pragma unroll
      for (int m = 0; m < NYW; ++m) s += P[Ly::y_w2 + m * NYW + q] * y2[m];
      t2[q] = f_tanh(s);
    }
    // reverse: y3 = (y2 + t2)/sqrt2, y2 = (y1 + t1)/sqrt2, y1 = res(y0, t0)
    T yb2[NYW], yb1[NYW], z[NYW];
#pragma unroll
    for (int q = 0; q < NYW; ++q) z[q] = ystb[q] * RSQ2 * (T(1) - t2[q] * t2[q]);
#pragma unroll
    for (int m = 0; m < NYW; ++m) {
      T s = ystb[m] * RSQ2;
#pragma unroll
      for (int q = 0; q < NYW; ++q) {
        s += P[Ly::y_w2 + m * NYW + q] * z[q];
        lds_add(&pg[Ly::y_w2 + m * NYW + q], y2[m] * z[q]);
      }
      yb2[m] = s;
    }
#pragma unroll
    for (int q = 0; q < NYW; ++q) lds_add(&pg[Ly::y_b2 + q], z[q]);
#pragma unroll
    for (int q = 0; q < NYW; ++q) z[q] = yb2[q] * RSQ2 * (T(1) - t1[q] * t1[q]);
#pragma unroll
    for (int m = 0; m < NYW; ++m) {
      T s = yb2[m] * RSQ2;
#pragma unroll
      for (int q = 0; q < NYW; ++q) {
        s += P[Ly::y_w1 + m * NYW + q] * z[q];
        lds_add(&pg[Ly::y_w1 + m * NYW + q], y1[m] * z[q]);
      }
      yb1[m] = s;
    }
#pragma unroll
    for (int q = 0; q < NYW; ++q) lds_add(&pg[Ly::y_b1 + q], z[q]);
#pragma unroll
    for (int q = 0; q < NYW; ++q) {
      z[q] = (DY0 == NYW ? yb1[q] * RSQ2 : yb1[q]) * (T(1) - t0[q] * t0[q]);
      lds_add(&pg[Ly::y_b0 + q], z[q]);
    }
#pragma unroll
    for (int m = 0; m < DY0; ++m)
#pragma unroll
      for (int q = 0; q < NYW; ++q) lds_add(&pg[Ly::y_w0 + m * NYW + q], y0[m] * z[q]);
  }
  __syncthreads();
  // ---------------------------------------------------------------- reverse: h stream (B2)
#pragma unroll
  for (int l = 2; l >= 0; --l) {
    const int d = l == 0 ? D0 : NH;
    const int DF = 3 * d + 2 * NH2, Q = DF / 4;
    const cptr<T> convw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2));
    const cptr<T> sngw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
    const int cw = l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2);
    const int cb = l == 0 ? Ly::conv_b0 : (l == 1 ? Ly::conv_b1 : Ly::conv_b2);
    const int sw = l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2);
    const int sb = l == 0 ? Ly::sng_b0 : (l == 1 ? Ly::sng_b1 : Ly::sng_b2);
    // single: s = tanh(c Ws + bs), h^{l+1} = res(h^l, s)
    for (int it = lane; it < nk * N * NH; it += 64) {
      const int kw = it / (N * NH), idx = it - kw * N * NH;
      T* sm = S(kw);
      const int i = idx / NH, f = idx - i * NH;
      const T s = sm[SM::sv + (l * N + i) * NH + f];
      const T sb_ = (d == NH) ? sm[SM::hb + idx] * RSQ2 : sm[SM::hb + idx];
      sm[SM::zs + idx] = sb_ * (T(1) - s * s);
    }
    __syncthreads();
    for (int it = lane; it < nk * Q * NH; it += 64) {
      const int kw = it / (Q * NH), idx = it - kw * Q * NH;
      T* sm = S(kw);
      T* pg = sm + SM::pg;
      const int q = idx / NH, f = idx - q * NH;
      T a = T(0), b = T(0);
      for (int i = 0; i < N; ++i) {
        a += sm[SM::cq + (l * N + i) * QM + q] * sm[SM::zs + i * NH + f];
        if (q == 0) b += sm[SM::zs + i * NH + f];
      }
      pg[sw + q * NH + f] += a;
      if (q == 0) pg[sb + f] += b;
    }
    for (int it = lane; it < nk * N * Q; it += 64) {
      const int kw = it / (N * Q), idx = it - kw * N * Q;
      T* sm = S(kw);
      const int i = idx / Q, q = idx - i * Q;
      T a = T(0);
#pragma unroll
      for (int f = 0; f < NH; ++f) a += sngw[q * NH + f] * sm[SM::zs + i * NH + f];
      const T c = sm[SM::cq + (l * N + i) * QM + q];
      const T z = a * (T(1) - c * c);
      sm[SM::zc + i * QM + q] = z;
      sm[SM::pg + cb + i * Q + q] += z;
    }
    __syncthreads();
    // conv: c = tanh(0.25 sum_j F_j w_j + b)
    for (int it = lane; it < nk * N * DF; it += 64) {
      const int kw = it / (N * DF), idx = it - kw * N * DF;
      T* sm = S(kw);
      const T* h = sm + SM::hl + SM::hoff(l);
      const T* g1 = sm + SM::g1 + l * 2 * D0;
      const int i = idx / DF, j = idx - i * DF;
      T F;
      if (j < d) F = h[i * d + j];
      else if (j < 3 * d) F = g1[((j - d) / d) * D0 + (j - d) % d];
      else F = sm[SM::g2 + ((l * 2 + (j - 3 * d) / 4) * N + i) * 4 + ((j - 3 * d) & 3)];
      const T z = T(0.25) * sm[SM::zc + i * QM + j / 4];
      sm[SM::pg + cw + i * DF + j] += z * F;
      sm[SM::fb + i * SM::DFM + j] = z * convw[i * DF + j];
    }
    __syncthreads();
    // inputs: h^l (direct + group means), g2 column means
    for (int it = lane; it < nk * 2 * N * NH2; it += 64) {
      const int kw = it / (2 * N * NH2), idx = it - kw * 2 * N * NH2;
      T* sm = S(kw);
      const int G = idx / (N * NH2), rem = idx - G * N * NH2, i = rem / NH2, f = rem - i * NH2;
      sm[SM::g2b + ((l * 2 + G) * N + i) * 4 + f] = sm[SM::fb + i * SM::DFM + 3 * d + 4 * G + f];
    }
    if (l > 0) {
      for (int it = lane; it < nk * N * NH; it += 64) {
        const int kw = it / (N * NH), idx = it - kw * N * NH;
        T* sm = S(kw);
        const T* fb = sm + SM::fb;
        const int k = idx / NH, m = idx - k * NH;
        const int G = k >= nup ? 1 : 0;
        T a = fb[k * SM::DFM + m] + ((d == NH) ? sm[SM::hb + idx] * RSQ2 : T(0));
        T s = T(0);
        for (int i = 0; i < N; ++i) s += fb[i * SM::DFM + d + G * d + m];
        sm[SM::hn + idx] = a + s * gw[G];
      }
    }
    __syncthreads();
    if (l > 0)
      for (int it = lane; it < nk * N * NH; it += 64) {
        const int kw = it / (N * NH), idx = it - kw * N * NH;
        S(kw)[SM::hb + idx] = S(kw)[SM::hn + idx];
      }
    __syncthreads();
  }
  // ---------------------------------------------------------------- reverse: pair stream (B3) + e-e Jastrow
  for (int it = lane; it < nk * N * N; it += 64) {
    const int kw = it / (N * N), idx = it - kw * N * N;
    T* sm = S(kw);
    T* pg = sm + SM::pg;
    const T* xs = sm + SM::xs;
    const int k = idx / N, i = idx - k * N;
    const bool diag = k == i;
    const int G = k >= nup ? 1 : 0;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = xs[3 * i + c] - xs[3 * k + c];
    const T r = f_sqrt(diag ? T(1) : d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    T p0[4] = {diag ? T(0) : r, diag ? T(0) : d[0], diag ? T(0) : d[1], diag ? T(0) : d[2]};
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
    T P2b[4], z2[4], P1b[4], z1[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) P2b[f] = sm[SM::g2b + ((2 * 2 + G) * N + i) * 4 + f] * gw[G];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      z2[o] = P2b[o] * RSQ2 * (T(1) - t2[o] * t2[o]);
      lds_add(&pg[Ly::dbl_b1 + o], z2[o]);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T s = sm[SM::g2b + ((1 * 2 + G) * N + i) * 4 + m] * gw[G] + P2b[m] * RSQ2;
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        s += P[Ly::dbl_w1 + m * 4 + o] * z2[o];
        lds_add(&pg[Ly::dbl_w1 + m * 4 + o], p1[m] * z2[o]);
      }
      P1b[m] = s;
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      z1[o] = P1b[o] * RSQ2 * (T(1) - t1[o] * t1[o]);
      lds_add(&pg[Ly::dbl_b0 + o], z1[o]);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int o = 0; o < 4; ++o) lds_add(&pg[Ly::dbl_w0 + m * 4 + o], p0[m] * z1[o]);
    if (k < i && !phg) {   // Jastrow.py:23-52: cusp r / (1 + alpha r), alpha per unordered pair
      const T cusp = P[Ly::jee_c + k * N + i], al = P[Ly::jee_a + k * N + i];
      const T den = al * r + T(1);
      pg[Ly::jee_a + k * N + i] += -cusp * r * r / (den * den);
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- outputs
  for (int it = lane; it < nk * Ly::total; it += 64) {
    const int kw = it / Ly::total, idx = it - kw * Ly::total;
    ((T*)ka.grad)[(size_t)(conf0 + kw) * Ly::total + idx] = S(kw)[SM::pg + idx];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k < nk && lane == 0) {
      const T lpsi = logdet[k] + (S(k)[SM::red] + S(k)[SM::red + 1]);
      if (ka.logabs) ((T*)ka.logabs)[conf0 + k] = lpsi;
      if (ka.phase) ((T*)ka.phase)[conf0 + k] = f_atan2(phi[k], phr[k]);
    }
  }
}

// out[j] = sum_b w[b] O[b][j] over the kernel layout, deterministic, in two launches:
// k_grad_partial: block (x, c) sums walkers [c*GR_CH, (c+1)*GR_CH) of columns 64x .. 64x+63
// (four waves stride the chunk, combined in wave order) -> part[c][j];
// k_grad_final: out[j] = sum_c part[c][j] in chunk order.  (One block per 64 columns over all
// walkers took 261 us for B = 4096 and 12 blocks; the chunked form fills the chip.)
constexpr int GR_CH = 64;
template <typename T>
__global__ __launch_bounds__(256) void k_grad_partial(const T* __restrict__ O, const T* __restrict__ w, int B, int n,
                                                      T* __restrict__ part) {
  __shared__ T ps[4][64];
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int s = threadIdx.x >> 6;
  const int b0 = blockIdx.y * GR_CH, b1 = b0 + GR_CH < B ? b0 + GR_CH : B;
  T a = T(0), a1 = T(0);
  if (j < n) {
    int b = b0 + s;
    for (; b + 4 < b1; b += 8) {
      a += w[b] * O[(size_t)b * n + j];
      a1 += w[b + 4] * O[(size_t)(b + 4) * n + j];
    }
    if (b < b1) a += w[b] * O[(size_t)b * n + j];
  }
  ps[s][threadIdx.x & 63] = a + a1;
  __syncthreads();
  if (s == 0 && j < n)
    part[(size_t)blockIdx.y * n + j] = (ps[0][threadIdx.x] + ps[1][threadIdx.x]) + (ps[2][threadIdx.x] + ps[3][threadIdx.x]);
}
template <typename T>
__global__ __launch_bounds__(256) void k_grad_final(const T* __restrict__ part, int nchunk, int n, T* __restrict__ out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  T a[4] = {T(0), T(0), T(0), T(0)};
  int c = 0;
  for (; c + 3 < nchunk; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += part[(size_t)(c + u) * n + j];
  }
  for (; c < nchunk; ++c) a[0] += part[(size_t)c * n + j];
  out[j] = (a[0] + a[1]) + (a[2] + a[3]);
}

// Kernel layout -> canonical (tree_flatten) order for `rows` gradient vectors.  map[k] >= 0: the
// kernel entry of canonical parameter k; -1: unused by the network (eplion, mu, nu, envelope.py);
// <= -2: the y coefficient W_y[m][c] (m*N + c = -2 - map[k]), whose kernel entry is the
// row-normalised What = W / |W_m| (nn.py:449-451): dW = (dWhat - What (What . dWhat)) / |W_m|.
template <typename T>
__global__ __launch_bounds__(256) void k_grad_canon(const T* __restrict__ G, int nkern, const int* __restrict__ map,
                                                    int ncanon, const T* __restrict__ what, int wy_off,
                                                    const double* __restrict__ wnorm, int N, int rows,
                                                    T* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)rows * ncanon) return;
  const int row = (int)(t / ncanon), k = (int)(t - (size_t)row * ncanon);
  const T* g = G + (size_t)row * nkern;
  const int m_ = map[k];
  T v = T(0);
  if (m_ >= 0) {
    v = g[m_];
  } else if (m_ <= -2) {
    const int mc = -2 - m_, m = mc / N;
    T dot = T(0);
    for (int cc = 0; cc < N; ++cc) dot += what[m * N + cc] * g[wy_off + m * N + cc];
    v = (g[wy_off + mc] - what[mc] * dot) / (T)wnorm[m];
  }
  out[t] = v;
}

}  // namespace aq
