// shape.hip -- kernels and host helpers for ONE (N, A) shape.  Compiled once
// per entry of AIQMC_SHAPE_LIST with -DAQ_N=<N> -DAQ_A=<A> (parallel build).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "ctx.h"
#include "walker_lap.h"
#include "quad_small.h"
#include "walker_pgrad.h"

using namespace aq;

#ifndef AQ_N
#error "compile with -DAQ_N=<electrons> -DAQ_A=<atoms>"
#endif

static int fail(int code, const std::string& m) { return aiqmc_fail(code, m); }

// One thread per (walker b, electron i): the acceptance of walkers_update (VMCmcstep.py:80-106)
// for the last sweep of aiqmc_mc_step (earlier sweeps fuse it into the next walker launch) and
// for the DMC drift-diffusion step.
template <typename T, int N>
__global__ __launch_bounds__(256) void k_accept(T* __restrict__ pos, AccArgs a, int B) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  // limdrift factors: every lane of the (full, 256-thread) block's waves before any returns
  const T te1 = taueff_wave<T>(a.taueff, a.tacc, 0, a.tstep, a.tpart), te2 = taueff_wave<T>(a.taueff, a.tacc, 1, a.tstep, a.tpart);
  // the next mc_step call's accumulator bank (not read by this call)
  for (int k = t; k < a.nzero; k += gridDim.x * blockDim.x) a.zero[k] = 0ull;
  if (t >= B * N) return;
  const int b = t / N, i = t - b * N;
  T xn[3];
  if (accept_one<T, N>(a, pos, b, i, xn, te1, te2)) {
#pragma unroll
    for (int c = 0; c < 3; ++c) pos[(size_t)b * 3 * N + 3 * i + c] = xn[c];
    if (a.count) atomicAdd(&a.count[b], 1);
  }
}

template <int N, int A>
static void pack_params(const aiqmc_ctx* c, const double* flat, std::vector<double>& out) {
  using Ly = Lay<N, A>;
  out.assign(Ly::total_ext, 0.0);
  const double* p = flat;
  auto take = [&](int n) {
    const double* q = p;
    p += n;
    return q;
  };
  // envelope[i]: alpha, beta, eplion, mu, nu, pi, sigma, xi (sorted keys)
  for (int i = 0; i < N; ++i) {
    const double* alpha = take(1);
    const double* beta = take(A);
    take(3 * A);   // eplion (unused by envelope.apply)
    take(A);       // mu
    take(A);       // nu
    const double* pi = take(3 * A);
    const double* sigma = take(3 * A);
    const double* xi = take(1);
    out[Ly::env_alpha + i] = alpha[0];
    out[Ly::env_xi + i] = xi[0];
    for (int a = 0; a < A; ++a) {
      out[Ly::env_beta + i * A + a] = beta[a];
      for (int d = 0; d < 3; ++d) {
        out[Ly::env_pi + (i * A + a) * 3 + d] = pi[a * 3 + d];
        out[Ly::env_sigma + (i * A + a) * 3 + d] = sigma[a * 3 + d];
      }
    }
  }
  const double* jae = take(N * A);
  for (int k = 0; k < N * A; ++k) out[Ly::jae_b + k] = jae[k];
  const double* ee_anti = take(c->nanti);
  const double* ee_par = take(c->npar);
  for (int q = 0; q < c->npar; ++q) {
    const int i = c->par[q], j = c->par[c->npar + q];
    out[Ly::jee_c + i * N + j] = out[Ly::jee_c + j * N + i] = 0.25;
    out[Ly::jee_a + i * N + j] = out[Ly::jee_a + j * N + i] = ee_par[q];
  }
  for (int q = 0; q < c->nanti; ++q) {
    const int i = c->anti[q], j = c->anti[c->nanti + q];
    out[Ly::jee_c + i * N + j] = out[Ly::jee_c + j * N + i] = 0.5;
    out[Ly::jee_a + i * N + j] = out[Ly::jee_a + j * N + i] = ee_anti[q];
  }
  // layers.input = {} ; layers.streams[l] = {convolutional{b,w}, double{b,w}, single{b,w}}
  const int D[3] = {Ly::D0, Ly::D1, Ly::D1};
  const int Q[3] = {Ly::Q0, Ly::Q1, Ly::Q1};
  const int cw[3] = {Ly::conv_w0, Ly::conv_w1, Ly::conv_w2};
  const int cb[3] = {Ly::conv_b0, Ly::conv_b1, Ly::conv_b2};
  const int sw[3] = {Ly::sng_w0, Ly::sng_w1, Ly::sng_w2};
  const int sb[3] = {Ly::sng_b0, Ly::sng_b1, Ly::sng_b2};
  const int dw[2] = {Ly::dbl_w0, Ly::dbl_w1};
  const int db[2] = {Ly::dbl_b0, Ly::dbl_b1};
  for (int l = 0; l < 3; ++l) {
    const double* b = take(N * Q[l]);
    const double* w = take(N * D[l]);
    for (int k = 0; k < N * Q[l]; ++k) out[cb[l] + k] = b[k];
    for (int k = 0; k < N * D[l]; ++k) out[cw[l] + k] = w[k];
    if (l < 2) {
      const double* bb = take(NH2);
      const double* ww = take(NH2 * NH2);
      for (int k = 0; k < NH2; ++k) out[db[l] + k] = bb[k];
      for (int k = 0; k < NH2 * NH2; ++k) out[dw[l] + k] = ww[k];
    }
    const double* sbp = take(NH);
    const double* swp = take(Q[l] * NH);
    for (int k = 0; k < NH; ++k) out[sb[l] + k] = sbp[k];
    for (int k = 0; k < Q[l] * NH; ++k) out[sw[l] + k] = swp[k];
  }
  // lane-order copies of the h-stream weights (layout.h x* blocks)
  for (int l = 0; l < 3; ++l) {
    const int QF = Q[l] / 4;
    for (int i = 0; i < N; ++i)
      for (int f = 0; f < 4; ++f) {
        for (int q = 0; q < Q[l]; ++q) out[Ly::xcw(l) + (i * 4 + f) * Ly::XQ + q] = out[cw[l] + i * D[l] + 4 * q + f];
        for (int s4 = 0; s4 < QF; ++s4) out[Ly::xcb(l) + (i * 4 + f) * Ly::XB + s4] = out[cb[l] + i * Q[l] + 4 * s4 + f];
        for (int q = 4 * QF; q < Q[l]; ++q) out[Ly::xcb(l) + (i * 4 + f) * Ly::XB + QF + q - 4 * QF] = out[cb[l] + i * Q[l] + q];
      }
    for (int f = 0; f < 4; ++f)
      for (int q = 0; q < Q[l]; ++q) out[Ly::xsw(l) + f * Ly::XQ + q] = out[sw[l] + q * NH + f];
    for (int q = 0; q < Q[l]; ++q)
      for (int f = 0; f < 4; ++f) out[Ly::xsr(l) + q * 4 + f] = out[sw[l] + q * NH + f];
  }
  // layers.streams_y[l].single_Ynlm {b, w}
  const int yin[3] = {Ly::DY0, NYW, NYW};
  const int yw[3] = {Ly::y_w0, Ly::y_w1, Ly::y_w2};
  const int yb[3] = {Ly::y_b0, Ly::y_b1, Ly::y_b2};
  for (int l = 0; l < 3; ++l) {
    const double* b = take(NYW);
    const double* w = take(yin[l] * NYW);
    for (int k = 0; k < NYW; ++k) out[yb[l] + k] = b[k];
    for (int k = 0; k < yin[l] * NYW; ++k) out[yw[l] + k] = w[k];
  }
  // orbitals[s] {b [2N], w [4][2N]} ; complex = even + i odd (nn.py:456)
  for (int s = 0; s < 2; ++s) {
    const double* b = take(2 * N);
    const double* w = take(NH * 2 * N);
    for (int col = 0; col < N; ++col) {
      out[Ly::orb_b + (s * N + col) * 2 + 0] = b[2 * col];
      out[Ly::orb_b + (s * N + col) * 2 + 1] = b[2 * col + 1];
      for (int f = 0; f < NH; ++f) {
        out[Ly::orb_w + ((s * NH + f) * N + col) * 2 + 0] = w[f * 2 * N + 2 * col];
        out[Ly::orb_w + ((s * NH + f) * N + col) * 2 + 1] = w[f * 2 * N + 2 * col + 1];
      }
    }
  }
  // y[0].w [6][N], row-normalised (nn.py:449-451)
  const double* wy = take(NYW * N);
  for (int m = 0; m < NYW; ++m) {
    double nrm = 0.0;
    for (int col = 0; col < N; ++col) nrm += wy[m * N + col] * wy[m * N + col];
    nrm = std::sqrt(nrm);
    for (int col = 0; col < N; ++col) out[Ly::wy + m * N + col] = wy[m * N + col] / nrm;
  }
  // system constants
  for (int a = 0; a < A; ++a) {
    for (int d = 0; d < 3; ++d) out[Ly::atoms + a * 3 + d] = c->atoms[a * 3 + d];
    out[Ly::charges + a] = c->charges[a];
    out[Ly::c34 + a] = std::pow(2.0 * c->charges[a], 0.75);
    out[Ly::c14 + a] = std::pow(2.0 * c->charges[a], 0.25);
  }
  double vnn = 0.0;
  for (int a = 0; a < A; ++a)
    for (int b = a + 1; b < A; ++b) {
      double r2 = 0.0;
      for (int d = 0; d < 3; ++d) {
        const double t = c->atoms[a * 3 + d] - c->atoms[b * 3 + d];
        r2 += t * t;
      }
      vnn += c->charges[a] * c->charges[b] / std::sqrt(r2);
    }
  out[Ly::vnn] = vnn;
}

// Canonical (tree_flatten) index -> kernel-layout index of the same parameter, the transpose of
// pack_params (see k_grad_canon for the -1 / <= -2 codes).
template <int N, int A>
static void gmap_impl(const aiqmc_ctx* c, std::vector<int>& map) {
  using Ly = Lay<N, A>;
  map.clear();
  auto put = [&](int k) { map.push_back(k); };
  for (int i = 0; i < N; ++i) {
    put(Ly::env_alpha + i);
    for (int a = 0; a < A; ++a) put(Ly::env_beta + i * A + a);
    for (int k = 0; k < 3 * A; ++k) put(-1);   // eplion
    for (int k = 0; k < A; ++k) put(-1);       // mu
    for (int k = 0; k < A; ++k) put(-1);       // nu
    for (int k = 0; k < 3 * A; ++k) put(Ly::env_pi + i * A * 3 + k);
    for (int k = 0; k < 3 * A; ++k) put(Ly::env_sigma + i * A * 3 + k);
    put(Ly::env_xi + i);
  }
  for (int k = 0; k < N * A; ++k) put(Ly::jae_b + k);
  auto pairs = [&](const std::vector<int>& t, int n) {
    for (int q = 0; q < n; ++q) {
      const int i = t[q], j = t[n + q];
      put(Ly::jee_a + (i < j ? i * N + j : j * N + i));
    }
  };
  pairs(c->anti, c->nanti);
  pairs(c->par, c->npar);
  const int D[3] = {Ly::D0, Ly::D1, Ly::D1};
  const int Q[3] = {Ly::Q0, Ly::Q1, Ly::Q1};
  const int cw[3] = {Ly::conv_w0, Ly::conv_w1, Ly::conv_w2};
  const int cb[3] = {Ly::conv_b0, Ly::conv_b1, Ly::conv_b2};
  const int sw[3] = {Ly::sng_w0, Ly::sng_w1, Ly::sng_w2};
  const int sb[3] = {Ly::sng_b0, Ly::sng_b1, Ly::sng_b2};
  const int dw[2] = {Ly::dbl_w0, Ly::dbl_w1};
  const int db[2] = {Ly::dbl_b0, Ly::dbl_b1};
  for (int l = 0; l < 3; ++l) {
    for (int k = 0; k < N * Q[l]; ++k) put(cb[l] + k);
    for (int k = 0; k < N * D[l]; ++k) put(cw[l] + k);
    if (l < 2) {
      for (int k = 0; k < NH2; ++k) put(db[l] + k);
      for (int k = 0; k < NH2 * NH2; ++k) put(dw[l] + k);
    }
    for (int k = 0; k < NH; ++k) put(sb[l] + k);
    for (int k = 0; k < Q[l] * NH; ++k) put(sw[l] + k);
  }
  const int yin[3] = {Ly::DY0, NYW, NYW};
  const int yw[3] = {Ly::y_w0, Ly::y_w1, Ly::y_w2};
  const int yb[3] = {Ly::y_b0, Ly::y_b1, Ly::y_b2};
  for (int l = 0; l < 3; ++l) {
    for (int k = 0; k < NYW; ++k) put(yb[l] + k);
    for (int k = 0; k < yin[l] * NYW; ++k) put(yw[l] + k);
  }
  for (int sp = 0; sp < 2; ++sp) {
    for (int k = 0; k < 2 * N; ++k) put(Ly::orb_b + (sp * N + k / 2) * 2 + (k & 1));
    for (int k = 0; k < NH * 2 * N; ++k) {
      const int f = k / (2 * N), r = k - f * 2 * N;
      put(Ly::orb_w + ((sp * NH + f) * N + r / 2) * 2 + (r & 1));
    }
  }
  for (int k = 0; k < NYW * N; ++k) put(-2 - k);
}

template <int N, int A>
static int set_lds_impl() {
  const int sizes[6] = {Smem<float, N, false>::bytes,  Smem<float, N, true>::bytes,  Smem<double, N, false>::bytes,
                        Smem<double, N, true>::bytes,  SmemRev<float, N, A>::bytes, SmemRev<double, N, A>::bytes};
  const void* fns[6] = {(const void*)&k_walker<float, N, A, MODE_GRAD>,  (const void*)&k_walker<float, N, A, MODE_LAP>,
                        (const void*)&k_walker<double, N, A, MODE_GRAD>, (const void*)&k_walker<double, N, A, MODE_LAP>,
                        (const void*)&k_walker_rev<float, N, A>,         (const void*)&k_walker_rev<double, N, A>};
  for (int k = 0; k < 6; ++k) {
    if (sizes[k] > 65536) {
      hipError_t e = hipFuncSetAttribute(fns[k], hipFuncAttributeMaxDynamicSharedMemorySize, sizes[k]);
      if (e != hipSuccess) return fail(AIQMC_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
    }
  }
  {   // proposal launches: RevWpb configurations per workgroup
    const int pb = RevWpb<float, true>::value * SmemRev<float, N, A, kFwdReg>::bytes;
    if (pb > 65536) {
      hipError_t e = hipFuncSetAttribute((const void*)&k_walker_rev<float, N, A, false, true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, pb);
      if (e != hipSuccess) return fail(AIQMC_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
    }
  }
  return 0;
}

// MODE_GRAD -> reverse-mode value+gradient kernel (walker_rev.h); MODE_LAP -> forward
// Laplacian kernel (walker_kernel.h); MODE_GRAD_FWD -> forward-mode gradient (diagnostics).
// proposal-launch grid: ceil(nconf / wpb) workgroups, padded to a multiple of the 8 XCDs so that
// xcd_major keeps each walker's proposals on one XCD (the padding workgroups exit at once)
static inline unsigned prop_blocks(int nconf, int wpb) {
  const unsigned nb = (unsigned)((nconf + wpb - 1) / wpb);
  return wpb > 1 ? (nb + 7u) & ~7u : nb;
}

// single-electron-moved configurations from the walker cache (quad_small.h): value only (pp
// quadrature, N <= 8) or value + gradient (Metropolis proposals and walker launches, N <= 4),
// several configurations per wave
// AIQMC_WALK_SPLIT=0 keeps small-batch walker launches on one wave per walker (A/B timing)
static bool walk_split_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("AIQMC_WALK_SPLIT");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}
// AIQMC_QUAD_GRAD=0 routes the packed proposals of 5 <= N <= 8 back to k_walker_rev (A/B timing)
static bool quad_grad_off() {
  static const int off = [] {
    const char* e = std::getenv("AIQMC_QUAD_GRAD");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return off != 0 && AQ_N > 4;
}

template <typename T, int N, int A>
static bool quad_small(const KArgs& ka, int nconf, hipStream_t s) {
  if constexpr (N <= 8) {   // pp quadrature: 4 (N <= 4) or 2 (N <= 8) configurations per wave
    if (ka.proposal && ka.ecache && ka.value_only && !ka.orb) {
      k_quad_value<T, N, A><<<dim3(prop_blocks(nconf, QSlot<N>::NSL)), dim3(64), 0, s>>>(ka);
      return true;
    }
  }
  if constexpr (N <= 8) {   // Metropolis proposals: 4 (N <= 4) or 2 (N <= 8) configurations per wave
    if (ka.proposal && ka.ecache && !ka.value_only && !ka.orb && !ka.ablate && !quad_grad_off()) {
      k_quad_grad<T, N, A><<<dim3((nconf + QSlot<N>::NSL - 1) / QSlot<N>::NSL), dim3(64), 0, s>>>(ka);
      return true;
    }
  }
  if constexpr (N <= 8) {   // walker launches: 4 (N <= 4) or 2 (N <= 8) per wave
    if (!ka.proposal && ka.wcache && !ka.value_only && !ka.orb && !ka.lapcache && !ka.one_wave) {
      k_quad_grad<T, N, A, true><<<dim3((nconf + QSlot<N>::NSL - 1) / QSlot<N>::NSL), dim3(64), 0, s>>>(ka);
      return true;
    }
  }
  return false;
}

// fp32 N2 proposals of small batches (the per-rank share of a strong-scaling run): the PW7
// instantiation (7 waves/SIMD, compact LDS; walker_rev.h) when it needs fewer rounds of waves than
// the 5-wave one and the batch takes at most three of those.  Measured slower at every batch size
// (N2, 512 / 1024 / 2048 walkers: proposal launch 40.3 -> 43.8, 65.9 -> 74.5, 116.0 -> 130.2 us,
// profiles/r04_s8_ab_pw7.txt), so it is compiled only with -DAQ_PW7 (AIQMC_PW7=0 / 1 forces it
// off / on there).
#ifdef AQ_PW7
static bool use_pw7(int nconf) {
  static const int force = [] {
    const char* e = std::getenv("AIQMC_PW7");
    return e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  if (force >= 0) return force == 1;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  const long s5 = 20L * ncu, s7 = 28L * ncu;
  const long r5 = (nconf + s5 - 1) / s5, r7 = (nconf + s7 - 1) / s7;
  return r7 < r5 && r5 <= 3;
}
#endif

template <int N, int A>
static void walker_impl(int dtype, int mode, const KArgs& ka, int nconf, hipStream_t s) {
  if (mode == MODE_GRAD && (dtype == AIQMC_F32 ? quad_small<float, N, A>(ka, nconf, s) : quad_small<double, N, A>(ka, nconf, s)))
    return;
  if (dtype == AIQMC_F32) {
    if (mode == MODE_LAP)
      k_walker<float, N, A, MODE_LAP><<<dim3(nconf), dim3(64), Smem<float, N, true>::bytes, s>>>(ka);
    else if (mode == MODE_GRAD && ka.proposal && ka.ecache) {   // proposals from the walker cache
#ifdef AQ_PW7
      if constexpr (N == 14 && A == 2) {
        if (use_pw7(nconf)) {
          k_walker_rev<float, N, A, false, true, true><<<dim3(prop_blocks(nconf, RevWpb<float, true>::value)),
                                                        dim3(64 * RevWpb<float, true>::value),
                                                        RevWpb<float, true>::value * SmemRev<float, N, A, kFwdReg, true>::bytes,
                                                        s>>>(ka);
          return;
        }
      }
#endif
      k_walker_rev<float, N, A, false, true><<<dim3(prop_blocks(nconf, RevWpb<float, true>::value)),
                                              dim3(64 * RevWpb<float, true>::value),
                                              RevWpb<float, true>::value * SmemRev<float, N, A, kFwdReg>::bytes, s>>>(ka);
    }
    else if (mode == MODE_GRAD && ka.walk_split && !ka.proposal && !ka.value_only && walk_split_on())
      k_walker_rev<float, N, A, false, false, false, false, true><<<dim3(nconf), dim3(128), SmemRev<float, N, A>::bytes,
                                                                  s>>>(ka);
    else if (mode == MODE_GRAD)
      k_walker_rev<float, N, A><<<dim3((nconf + RevWpb<float, false>::value - 1) / RevWpb<float, false>::value),
                                  dim3(64 * RevWpb<float, false>::value),
                                  RevWpb<float, false>::value * SmemRev<float, N, A>::bytes, s>>>(ka);
    else
      k_walker<float, N, A, MODE_GRAD><<<dim3(nconf), dim3(64), Smem<float, N, false>::bytes, s>>>(ka);
  } else {
    if (mode == MODE_LAP)
      k_walker<double, N, A, MODE_LAP><<<dim3(nconf), dim3(64), Smem<double, N, true>::bytes, s>>>(ka);
    else if (mode == MODE_GRAD && ka.proposal && ka.ecache)   // proposals from the walker cache
      k_walker_rev<double, N, A, false, true><<<dim3(prop_blocks(nconf, RevWpb<double, true>::value)),
                                              dim3(64 * RevWpb<double, true>::value),
                                              RevWpb<double, true>::value * SmemRev<double, N, A, kFwdReg>::bytes, s>>>(ka);
    else if (mode == MODE_GRAD)
      k_walker_rev<double, N, A><<<dim3(nconf), dim3(64), SmemRev<double, N, A>::bytes, s>>>(ka);
    else
      k_walker<double, N, A, MODE_GRAD><<<dim3(nconf), dim3(64), Smem<double, N, false>::bytes, s>>>(ka);
  }
}

// Local energy: adjoint pass (k_walker_rev<PREP>) then first-derivative pass (k_walker_lap).
// phase: the same pair for theta = arg psi (the PH instantiations, complex_output=True)
template <typename T, int N, int A, bool PH>
static void lap_launch(const KArgs& k1, const KArgs& k2, int nconf, int waves, hipStream_t s) {
  const dim3 wg(64 * waves);   // waves per walker in the first-derivative pass: 1, 2 or 4
  k_walker_rev<T, N, A, true, false, false, PH><<<dim3(nconf), dim3(64), SmemRev<T, N, A>::bytes, s>>>(k1);
  if (waves == 1)
    k_walker_lap<T, N, A, 1, PH><<<dim3(nconf), wg, SmemLap<T, N, A>::bytes, s>>>(k2);
  else
    k_walker_lap<T, N, A, 4, PH><<<dim3(nconf), wg, SmemLap<T, N, A>::bytes, s>>>(k2);
}
template <int N, int A>
static void lap_impl(int dtype, const KArgs& k1, const KArgs& k2, int nconf, int waves, int phase, hipStream_t s) {
  if (dtype == AIQMC_F32) {
    if (phase) lap_launch<float, N, A, true>(k1, k2, nconf, waves, s);
    else lap_launch<float, N, A, false>(k1, k2, nconf, waves, s);
  } else {
    if (phase) lap_launch<double, N, A, true>(k1, k2, nconf, waves, s);
    else lap_launch<double, N, A, false>(k1, k2, nconf, waves, s);
  }
}

template <int N, int A>
static void moved_impl(int dtype, const KArgs& ka, hipStream_t s) {
  if (ka.value_only && ka.xnew) {   // pp quadrature: values only, one configuration per lane
    const int nv = (ka.nconf + 63) / 64;
    if (dtype == AIQMC_F32)
      k_moved_value<float, N, A><<<dim3(prop_blocks(nv, MOVED_WPB)), dim3(64 * MOVED_WPB), 0, s>>>(ka);
    else
      k_moved_value<double, N, A><<<dim3(prop_blocks(nv, MOVED_WPB)), dim3(64 * MOVED_WPB), 0, s>>>(ka);
    return;
  }
  const int nb = (ka.nconf + 15) / 16;
  if (dtype == AIQMC_F32)
    k_moved_electron<float, N, A><<<dim3(prop_blocks(nb, MOVED_WPB)), dim3(64 * MOVED_WPB), 0, s>>>(ka);
  else
    k_moved_electron<double, N, A><<<dim3(prop_blocks(nb, MOVED_WPB)), dim3(64 * MOVED_WPB), 0, s>>>(ka);
}

template <int N, int A>
static void accept_impl(int dtype, void* pos, const AccArgs& a, int B, hipStream_t s) {
  const int nb = (B * N + 255) / 256;
  if (dtype == AIQMC_F32)
    k_accept<float, N><<<dim3(nb), dim3(256), 0, s>>>((float*)pos, a, B);
  else
    k_accept<double, N><<<dim3(nb), dim3(256), 0, s>>>((double*)pos, a, B);
}

// per-walker parameter gradients in the kernel layout: out [nconf][Lay::total]
template <typename T, int N, int A>
static int pgrad_launch(const KArgs& ka, int nconf, hipStream_t s) {
  constexpr int K = PgK<N>::value;   // walkers per wave (walker_pgrad.h)
  constexpr int bytes = K * SmemPG<T, N, A>::bytes;
  if (bytes > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)&k_param_grad<T, N, A, K>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return fail(AIQMC_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  k_param_grad<T, N, A, K><<<dim3((nconf + K - 1) / K), dim3(64), bytes, s>>>(ka);
  return 0;
}

template <int N, int A>
static int pgrad_impl(int dtype, const KArgs& ka, int nconf, hipStream_t s) {
  if (dtype == AIQMC_F32) {
    if (int rc = pgrad_launch<float, N, A>(ka, nconf, s)) return rc;
  } else {
    if (int rc = pgrad_launch<double, N, A>(ka, nconf, s)) return rc;
  }
  return 0;
}

static void phase_read_impl(unsigned long long* out) {
#ifdef AQ_PHASE_PROF
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(aq_phase_cycles), 32 * sizeof(unsigned long long));
  unsigned long long z[32] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(aq_phase_cycles), z, sizeof(z));
#else
  for (int k = 0; k < 32; ++k) out[k] = 0;
#endif
}

#define AQ_CAT2(a, b, c) aiqmc_shape_ops_##a##_##b##c
#define AQ_CAT(a, b) AQ_CAT2(a, b, )
bool AQ_CAT(AQ_N, AQ_A)(ShapeOps* ops) {
  ops->set_lds = &set_lds_impl<AQ_N, AQ_A>;
  ops->walker = &walker_impl<AQ_N, AQ_A>;
  ops->accept = &accept_impl<AQ_N, AQ_A>;
  ops->moved = &moved_impl<AQ_N, AQ_A>;
  ops->lap = &lap_impl<AQ_N, AQ_A>;
  ops->lcache_n = LapCache<AQ_N, AQ_A>::size;
  ops->phase_read = &phase_read_impl;
  ops->wcache_n = WCache<AQ_N, AQ_A>::size;
  ops->ecache_n = ECache<AQ_N, AQ_A>::size;
  ops->nkern = Lay<AQ_N, AQ_A>::total;
  ops->nprm = Lay<AQ_N, AQ_A>::total_ext;
  ops->ncanon = &Lay<AQ_N, AQ_A>::canon;
  ops->pack = &pack_params<AQ_N, AQ_A>;
  ops->gmap = &gmap_impl<AQ_N, AQ_A>;
  ops->pgrad = &pgrad_impl<AQ_N, AQ_A>;
  ops->wy_off = Lay<AQ_N, AQ_A>::wy;
  {
    constexpr int N = AQ_N, A = AQ_A;
    const int f[6] = {RevWpb<float, true>::value * SmemRev<float, N, A, kFwdReg>::bytes,
                      RevWpb<float, false>::value * SmemRev<float, N, A>::bytes, SmemRev<float, N, A>::bytes,
                      SmemLap<float, N, A>::bytes, PgK<N>::value * SmemPG<float, N, A>::bytes, Smem<float, N, true>::bytes};
    const int d[6] = {RevWpb<double, true>::value * SmemRev<double, N, A, kFwdReg>::bytes,
                      SmemRev<double, N, A>::bytes, SmemRev<double, N, A>::bytes, SmemLap<double, N, A>::bytes,
                      PgK<N>::value * SmemPG<double, N, A>::bytes, Smem<double, N, true>::bytes};
    const int wf[6] = {RevWpb<float, true>::value, RevWpb<float, false>::value, 1, 0, 1, 1};
    const int wd[6] = {RevWpb<double, true>::value, 1, 1, 0, 1, 1};
    for (int k = 0; k < 6; ++k) {
      ops->dyn_lds[0][k] = f[k];
      ops->dyn_lds[1][k] = d[k];
      ops->wg_waves[0][k] = wf[k];   // 0: the launch chooses (k_walker_lap: 1, 2 or 4 waves)
      ops->wg_waves[1][k] = wd[k];
    }
  }
  return true;
}
