// gj.h -- in-register complex Gauss-Jordan inverse + log|det| for one N x N
// matrix per wavefront (replaces jnp.linalg.slogdet, network_blocks.py:156, and
// provides B = A^{-1} for the derivative contractions).
//
// Layout: lane l = 16*cg + j holds row j (< N) of [A | I], columns
// cg*CW .. cg*CW+CW-1 (CW = ceil(2N/4)) in VGPRs for the whole elimination.
// Partial pivoting is virtual: at step k the pivot row p_k is the unused row
// with the first maximal |re|+|im| in column k (LAPACK izamax rule); no rows
// move.  With E the accumulated row operations, E A = L with L[p_k,k] = 1,
// so A^{-1}[k,:] = (right block)[p_k,:] and det A = sgn(p) prod_k pivot_k.
// Per step: one 16-lane DPP max + ballot for the pivot, 2 readlanes for the
// pivot value, 2 + 2*CW ds_bpermute broadcasts, CW complex row updates.
#pragma once
#include "jets.h"

namespace aq {

template <typename T> __device__ __forceinline__ T f_max(T a, T b) { return a > b ? a : b; }

template <typename T> __device__ __forceinline__ T rowmax16(T x) {
  x = f_max(x, dpp<0xB1>(x));
  x = f_max(x, dpp<0x4E>(x));
  x = f_max(x, dpp<0x141>(x));
  x = f_max(x, dpp<0x140>(x));
  return x;
}

// A[r][c] = Ph[r][c] * Yv[r][c]  (Ph complex interleaved [N][N][2], Yv real [N][N]).
// Writes B = A^{-1} to Bout[N][N][2]; returns log|det A| and the unit phase (phr, phi).
template <typename T, int N>
__device__ __forceinline__ void gj_inverse(const T* Ph, const T* Yv, T* Bout, int lane, T& logdet, T& phr,
                                           T& phi) {
  constexpr int CW = (2 * N + 3) / 4;
  const int j = lane & 15;
  const int cg = lane >> 4;
  const bool rowlive = j < N;
  T mr[CW], mi[CW];
#pragma unroll
  for (int t = 0; t < CW; ++t) {
    const int c = cg * CW + t;
    T a = T(0), b = T(0);
    if (rowlive && c < N) {
      const T y = Yv[j * N + c];
      a = Ph[(j * N + c) * 2] * y;
      b = Ph[(j * N + c) * 2 + 1] * y;
    } else if (rowlive && c < 2 * N && c - N == j) {
      a = T(1);
    }
    mr[t] = a;
    mi[t] = b;
  }
  bool used = !rowlive;
  int myk = 0;
  int pk[N];
  T ld = T(0), pr_ = T(1), pi_ = T(0);
#pragma unroll
  for (int k = 0; k < N; ++k) {
    constexpr int dummy = 0;
    (void)dummy;
    const int kc = k / CW, kt = k % CW;
    const bool cand = (cg == kc) && !used;
    const T key = cand ? f_abs(mr[kt]) + f_abs(mi[kt]) : T(-1);
    const T m = rowmax16(key);
    const unsigned long long mask = __ballot(cand && key == m);
    const int p = (int)__builtin_ctzll(mask) - 16 * kc;
    pk[k] = p;
    if (j == p) {
      used = true;
      myk = k;
    }
    const T pr = rdlane(mr[kt], 16 * kc + p);
    const T pim = rdlane(mi[kt], 16 * kc + p);
    const T den = pr * pr + pim * pim;
    const T rden = f_rcp(den);
    ld += T(0.5) * f_log(den);                 // log|pivot|
    {
      const T rm = f_sqrt(rden);
      const T ur = pr * rm, ui = pim * rm;
      const T nr = pr_ * ur - pi_ * ui, ni = pr_ * ui + pi_ * ur;
      pr_ = nr;
      pi_ = ni;
    }
    const T ir = pr * rden, ii = -pim * rden;
    const T fr = __shfl(mr[kt], 16 * kc + j);
    const T fi = __shfl(mi[kt], 16 * kc + j);
    const bool isp = (j == p);
#pragma unroll
    for (int t = 0; t < CW; ++t) {
      const T qr = __shfl(mr[t], 16 * cg + p);
      const T qi = __shfl(mi[t], 16 * cg + p);
      const T sr = qr * ir - qi * ii, si = qr * ii + qi * ir;
      const T ur = mr[t] - (fr * sr - fi * si);
      const T ui = mi[t] - (fr * si + fi * sr);
      mr[t] = isp ? sr : ur;
      mi[t] = isp ? si : ui;
    }
  }
#pragma unroll
  for (int t = 0; t < CW; ++t) {
    const int c = cg * CW + t;
    if (rowlive && c >= N && c < 2 * N) {
      Bout[(myk * N + (c - N)) * 2] = mr[t];
      Bout[(myk * N + (c - N)) * 2 + 1] = mi[t];
    }
  }
  int inv = 0;
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int b = a + 1; b < N; ++b) inv += pk[a] > pk[b] ? 1 : 0;
  if (inv & 1) {
    pr_ = -pr_;
    pi_ = -pi_;
  }
  logdet = ld;
  phr = pr_;
  phi = pi_;
}

}  // namespace aq
