// electron.h -- the per-electron stage shared by both walker kernels.
//
// Every lane evaluates, for its electron le = min(lane & 15, N-1) and along its
// own coordinate direction x_{le,lc} (value row lc = 3: no direction), the
// quantities that depend on x_le only:
//   ae features [r_ia, x_i - R_a] (nn.py:125-137)          -> hf[4A]
//   Ylm stream input + three tanh/residual layers           -> yst[6]
//     (nn.py:156-193, 313-341; Q3: x[3] reads x[2]; Q4: unit-vector inputs)
//   envelope of row le (envelope.py:26-30, Q1)              -> env
//   e-n Pade Jastrow of electron le (Jastrow.py:84-93)      -> jae
//   e-n potential -sum_a Z_a / r_ia (hamiltonian.py:190-198) -> ven
// as second-order forward jets PJ {v, d1, d2}.
#pragma once
#include "jets.h"
#include "layout.h"

namespace aq {

template <typename T> __device__ __forceinline__ PJ<T> pj_recip(PJ<T> a) {
  const T q = f_rcp(a.v);
  const T q2 = q * q;
  return PJ<T>{q, -a.d1 * q2, (T(2) * a.d1 * a.d1 * q - a.d2) * q2};
}

template <typename T, int A>
struct ElecOut {
  PJ<T> hf[4 * A];
  PJ<T> yst[NYW];
  PJ<T> env, jae;
  T ven;
};

// xpos: the 3 coordinates of electron le; le selects the per-electron parameters.
template <typename T, int N, int A>
__device__ __forceinline__ void electron_stage(cptr<T> P, const T* xpos, int le, int lc,
                                               ElecOut<T, A>& o) {
  using Ly = Lay<N, A>;
  PJ<T> xe[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) xe[c] = PJ<T>{xpos[c], (lc == c) ? T(1) : T(0), T(0)};
  PJ<T> yin[4 * A + 2];
  PJ<T> ra[A];
  PJ<T> aev[A][3];
  PJ<T> hisum = pjc(T(0)), spsum = pjc(T(0));
  o.ven = T(0);
  const T PI = T(3.141592653589793);
  const T c0 = T(0.5) * f_sqrt(T(1) / PI), c1 = f_sqrt(T(3) / (T(4) * PI));
  const T k15h = T(0.5) * f_sqrt(T(15) / PI), k5q = T(0.25) * f_sqrt(T(5) / PI);
  const T k15q = T(0.25) * f_sqrt(T(15) / PI), k35 = T(0.25) * f_sqrt(T(35) / (T(2) * PI));
  const T k105h = T(0.5) * f_sqrt(T(105) / PI), k21 = T(0.25) * f_sqrt(T(21) / (T(2) * PI));
  const T k7 = T(0.25) * f_sqrt(T(7) / PI), k105q = T(0.25) * f_sqrt(T(105) / PI);
#pragma unroll
  for (int a = 0; a < A; ++a) {
    PJ<T> ae[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) ae[c] = xe[c] - P[Ly::atoms + a * 3 + c];     // nn.py:111
    const PJ<T> r = pj_sqrt(ae[0] * ae[0] + ae[1] * ae[1] + ae[2] * ae[2]);   // nn.py:113
    ra[a] = r;
#pragma unroll
    for (int c = 0; c < 3; ++c) aev[a][c] = ae[c];
    o.hf[4 * a] = r;                                                        // nn.py:134-136
#pragma unroll
    for (int c = 0; c < 3; ++c) o.hf[4 * a + 1 + c] = ae[c];
    const PJ<T> rinv = pj_recip(r);
    const PJ<T> x0 = ae[0] * rinv, x1 = ae[1] * rinv, x2 = ae[2] * rinv;   // t = ae / r (nn.py:327)
    yin[4 * a + 0] = pjc(c0);                                               // nn.py:164-167
    yin[4 * a + 1] = c1 * x0;
    yin[4 * a + 2] = c1 * x1;
    yin[4 * a + 3] = c1 * x2;
#pragma unroll
    for (int m = 0; m < 4; ++m) spsum = spsum + yin[4 * a + m];
    // nn.py:182-193 with y = r (Q4) and x[3] -> x[2] (Q3); the 5 d-terms share 1/y^2,
    // the 7 f-terms 1/y^3; only their sum enters (mean over all 12A terms, nn.py:336)
    const PJ<T> y2 = r * r;
    const PJ<T> inv2 = rinv * rinv, inv3 = inv2 * rinv;
    const PJ<T> x00 = x0 * x0, x11 = x1 * x1, x22 = x2 * x2;
    const PJ<T> x01 = x0 * x1;
    const PJ<T> s2 = k15h * x01 + k15h * (x1 * x2) + k5q * (T(3) * x22 - y2) + k15h * (x0 * x2) +
                     k15q * (x00 - x11);
    const PJ<T> f5 = T(5) * x22 - y2;
    const PJ<T> s3 = k35 * (x1 * (T(3) * x00 - x11)) + k105h * (x01 * x2) + k21 * (x1 * f5) +
                     k7 * (x2 * (T(5) * x22 - T(3) * y2)) + k21 * (x0 * f5) + k105q * ((x00 - x11) * x2) +
                     k35 * (x0 * (x00 - T(3) * x11));
    hisum = hisum + s2 * inv2 + s3 * inv3;
    o.ven -= P[Ly::charges + a] * rinv.v;                                    // hamiltonian.py:190-198
  }
  yin[4 * A] = hisum * (T(1) / T(12 * A));                                   // nn.py:336-339
  yin[4 * A + 1] = spsum * (T(1) / T(4 * A));
  // Ynlm stream (nn.py:313-319, 340-341)
  constexpr int DY0 = Ly::DY0;
#pragma unroll
  for (int q = 0; q < NYW; ++q) {
    PJ<T> s = P[Ly::y_w0 + q] * yin[0];
#pragma unroll
    for (int m = 1; m < DY0; ++m) s = s + P[Ly::y_w0 + m * NYW + q] * yin[m];
    o.yst[q] = pj_tanh(s + P[Ly::y_b0 + q]);
    if constexpr (DY0 == NYW) o.yst[q] = T(0.70710678118654752) * (yin[q] + o.yst[q]);
  }
#pragma unroll
  for (int l = 1; l < 3; ++l) {
    const int wo = l == 1 ? Ly::y_w1 : Ly::y_w2;
    const int bo = l == 1 ? Ly::y_b1 : Ly::y_b2;
    PJ<T> nx[NYW];
#pragma unroll
    for (int q = 0; q < NYW; ++q) {
      PJ<T> s = P[wo + q] * o.yst[0];
#pragma unroll
      for (int m = 1; m < NYW; ++m) s = s + P[wo + m * NYW + q] * o.yst[m];
      nx[q] = pj_tanh(s + P[bo + q]);
    }
#pragma unroll
    for (int q = 0; q < NYW; ++q) o.yst[q] = T(0.70710678118654752) * (o.yst[q] + nx[q]);
  }
  // envelope of row le (envelope.py:26-30) and e-n Jastrow (Jastrow.py:84-93)
  const T alpha = P[Ly::env_alpha + le], xi = P[Ly::env_xi + le];
  PJ<T> e1 = pjc(T(0)), e2 = pjc(T(0)), ja = pjc(T(0));
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const T beta = P[Ly::env_beta + le * A + a];
    e1 = e1 + alpha * pj_exp(-beta * (ra[a] * ra[a]));
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const T pi_ = P[Ly::env_pi + (le * A + a) * 3 + c];
      const T sg = P[Ly::env_sigma + (le * A + a) * 3 + c];
      e2 = e2 + (sg * xi) * pj_exp(-pi_ * aev[a][c]);
    }
    const T bj = P[Ly::jae_b + le * A + a];
    const T c34 = P[Ly::c34 + a], c14 = P[Ly::c14 + a];
    const PJ<T> ex = pj_exp(-(c14 * bj) * ra[a]);
    ja = ja + (-c34 * f_rcp(T(2) * bj)) * (pjc(T(1)) - ex);
  }
  o.env = e1 + e2;
  o.jae = ja;
}

}  // namespace aq
