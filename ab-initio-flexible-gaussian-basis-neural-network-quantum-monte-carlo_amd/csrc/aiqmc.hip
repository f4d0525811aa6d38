// aiqmc.hip -- MI355X (gfx950) AIQMC VMC inner loop: kernels + C-ABI.
//
// Entry points are declared in include/aiqmc.h (which cites the reference
// functions each one replaces).  Kernels:
//   k_walker<T,N,A,MODE>  one wavefront per configuration (walker_kernel.h)
//   k_taueff              device-batch reduction of |grad|^2 -> limdrift factor
//   k_accept              Metropolis acceptance + move (VMCmcstep.py:84-106)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "aiqmc.h"
#include "ctx.h"
#include "ecp.h"
#include "walker_pgrad.h"

using namespace aq;

// fp32 mc_step sums its limdrift reductions in the walker / proposal launches up to this many
// walkers per call (aiqmc_debug_set_fuse_reduce: 1 = by batch size, 2 = always, 0 = never).
// Round 4, with 256 accumulator slots: fused is as fast or faster at every measured size (N2 per
// iteration, launches vs fused: 4096 walkers 3.026-3.030 vs 2.993-3.000 ms), so no limit.
constexpr int FUSE_REDUCE_MAX_B = 1 << 30;

// ============================================================================ small kernels

// complex_output=True local energy from the log|psi| pass (e_re = E_L = V - (lap log|psi| +
// |grad log|psi||^2) / 2, ga = grad log|psi|) and the phase pass (gp = grad theta, lp = lap theta):
// hamiltonian.py:110-130,  KE = -1/2 [lap log|psi| + i lap theta] - 1/2 |ga|^2 + 1/2 |gp|^2 - i ga.gp
// ADD_IM: e_im already holds a part of the energy (the pp local energy's imaginary nonlocal part):
// the phase terms are added to it, and to e_re, directly (no complex-minus-real difference).
template <typename T, bool ADD_IM = false>
__global__ __launch_bounds__(256) void k_complex_el(int B, int n3, const T* __restrict__ ga, const T* __restrict__ gp,
                                                    const T* __restrict__ lp, T* __restrict__ e_re, T* __restrict__ e_im) {
  const int b = blockIdx.x * 256 + (int)threadIdx.x;
  if (b >= B) return;
  T pp = T(0), ap = T(0);
  for (int k = 0; k < n3; ++k) {
    const T p = gp[(size_t)b * n3 + k];
    pp += p * p;
    ap += ga[(size_t)b * n3 + k] * p;
  }
  e_re[b] += T(0.5) * pp;
  if (ADD_IM) e_im[b] += T(-0.5) * lp[b] - ap;
  else e_im[b] = T(-0.5) * lp[b] - ap;
}

// v2 = sum(x[0..n)) ; taueff = (sqrt(1 + 2 tau a v2) - 1)/(a v2), a = 0.25  (VMCmcstep.py:11-14)
// One 1024-thread block; thread t sums x[t + 1024 j] in 8 independent partial sums, 32 loads in
// flight per thread (n = B N = 57,344 takes two rounds; with 8 in flight it took 7 and the
// launch 4.8 us), then a fixed-order tree -- the result is deterministic.
template <typename T>
__global__ __launch_bounds__(1024) void k_taueff(const T* __restrict__ x, int n, double tstep, double* out) {
  __shared__ double red[1024];
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int i = threadIdx.x;
  for (; i + 31 * 1024 < n; i += 32 * 1024) {
    T v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = x[i + k * 1024];
#pragma unroll
    for (int k = 0; k < 32; ++k) s[k & 7] += (double)v[k];
  }
  for (; i + 7 * 1024 < n; i += 8 * 1024) {
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = x[i + k * 1024];
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += (double)v[k];
  }
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if (i + k * 1024 < n) s[k] += (double)x[i + k * 1024];
  red[threadIdx.x] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double v2 = red[0];
    const double a = 0.25;
    T v2t = (T)v2;
    T te = (sqrt((T)1 + (T)2 * (T)tstep * (T)a * v2t) - (T)1) / ((T)a * v2t);
    *out = (double)te;
  }
}

// fp32 limdrift reduction of an unfused sweep (aiqmc_debug_set_fuse_reduce(0)): TPART
// workgroups, every element entering as tacc_fix(x) -- the fused accumulators' arithmetic --
// each workgroup writing its exact integer partial sum to part[blockIdx.x]; the consumers
// (taueff_wave) add the TPART partials with one load per lane and form the factor themselves.
// The same bits as the fused path at any batch size and in any order; no atomics, fences or a
// finalising workgroup on the critical path (k_taueff, one 1024-thread workgroup, took 4.6 us for
// the N2 proposal batch; a 32-workgroup version finishing in its last workgroup 4.5 us).
// Each element enters through tacc_split (walker_kernel.h: lo / mid / hi / bad, exact; hi
// saturating), so non-finite and huge |grad|^2 reach the consumers as the fused path's do;
// part = this kind's [4][TPART] block (lo, mid, hi, bad per workgroup).
__global__ __launch_bounds__(256) void k_taueff_part(const float* __restrict__ x, int n,
                                                     unsigned long long* __restrict__ part) {
  __shared__ unsigned long long ws[4][4];
  unsigned long long v = 0, mid = 0, hi = 0, bad = 0;
  const int stride = TPART * 256;
  for (int i = blockIdx.x * 256 + (int)threadIdx.x; i < n; i += 8 * stride) {
    float t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = i + k * stride < n ? x[i + k * stride] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double d = (double)t[k];
      if (d >= 0.0 && d < 0x1p24) {
        v += tacc_fix(d);
      } else {
        const TFix f = tacc_split(d);
        v += f.lo;
        mid += f.mid;
        hi = sat_add_u64(hi, f.hi);
        bad += f.bad;
      }
    }
  }
  v = wave_sum_u64(v);
  mid = wave_sum_u64(mid);
  hi = wave_sum_sat_u64(hi);
  bad = wave_sum_u64(bad);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    ws[0][w] = v;
    ws[1][w] = mid;
    ws[2][w] = hi;
    ws[3][w] = bad;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const unsigned long long* q = ws[threadIdx.x];
    part[threadIdx.x * TPART + blockIdx.x] =
        threadIdx.x == 2 ? sat_add_u64(sat_add_u64(q[0], q[1]), sat_add_u64(q[2], q[3])) : (q[0] + q[1]) + (q[2] + q[3]);
  }
}

// Per-sweep random draws (production mode), one thread per (walker b, electron i):
// gauss1[b][3i..3i+2], gauss2[b][i][0..2] standard normals, u[b][i] in [0,1) --
// the same buffers the caller supplies in AIQMC_RNG_HOST mode.
template <typename T>
__global__ __launch_bounds__(256) void k_draws(uint64_t seed, uint64_t step, int B, int N, T* __restrict__ g1,
                                               T* __restrict__ g2, T* __restrict__ u) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * N) return;
  float a[3], b[3], c[4];
  philox_normal3f(seed, step, (uint32_t)t, 0u, a);
  philox_normal3f(seed, step, (uint32_t)t, 1u, b);
  philox_u4(seed, step, (uint32_t)t, 2u, c);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    g1[(size_t)t * 3 + k] = (T)a[k];
    g2[(size_t)t * 3 + k] = (T)b[k];
  }
  u[t] = (T)(c[0] - 5.9604644775390625e-08f);   // [0,1)
}

// DMC reductions run over DMC_NB blocks (partial sums / minima per block in a fixed order), then
// one thread combines the block results in block order: deterministic, and the chip is not
// reduced to one block (the single-block forms took 29 us (sum), 72 us (weights) at B = 4096).
constexpr int DMC_NB = 64;

// DMC drift-diffusion extras (DMC/drift_diffusion.py:15-22):
// grad != nullptr: out[0] = sum over all coordinates of the proposed configuration
//   x + limdrift(grad) tau + sqrt(tau) gauss1 (the `changed_configuration` of :66);
// grad == nullptr: out[1] = sum of x (after acceptance), out[2] = tdamp = out[1] / out[0].
// k_dmc_sum_part: part[blk] = this block's share; k_dmc_sum_fin: the sum of part[0..DMC_NB) in order.
template <typename T>
__global__ __launch_bounds__(256) void k_dmc_sum_part(const T* __restrict__ x, const T* __restrict__ grad,
                                                      const T* __restrict__ g1, const double* __restrict__ taueff,
                                                      double tstep_d, int n, double* __restrict__ part) {
  __shared__ double red[256];
  const T tstep = (T)tstep_d;
  const T sq = sqrt(tstep);
  const T te = grad ? (T)taueff[0] : T(0);
  double acc = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += 256 * DMC_NB) {
    T v = x[i];
    if (grad) v = v + (grad[i] * te * tstep + sq * g1[i]);
    acc += (double)v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void k_dmc_sum_fin(const double* __restrict__ part, int proposed, double* out) {
  if (threadIdx.x != 0) return;
  double a = 0.0;
  for (int b = 0; b < DMC_NB; ++b) a += part[b];
  if (proposed) {
    out[0] = a;
  } else {
    out[1] = a;
    out[2] = a / out[0];
  }
}

// Energy statistics of one iteration (loss.py:206-208 through constants.pmean_stats), one
// workgroup: out[0..3] = [sum |e - m|^2, n m, n m^2, n] in fp64 (m = the mean of these n
// energies; the summed 4-vector of all ranks gives the pooled mean and variance), and with
// finalize (one rank) out[4..5] = [m, sum |e - m|^2 / n], the reference's two-pass values.
// k_energy_stats_final forms them from a summed 4-vector after the all-reduce (Chan's
// combination; products not contracted into FMAs, so one rank's between-term n m^2 - n m^2 is 0).
__device__ __forceinline__ double block_sum_1024(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k];
  return t;
}
__device__ __forceinline__ void energy_stats_final(double* out) {
#pragma clang fp contract(off)
  const double mean = out[1] / out[3];
  double between = out[2] - out[3] * mean * mean;
  between = between > 0.0 ? between : 0.0;
  out[4] = mean;
  out[5] = (out[0] + between) / out[3];
}
template <typename T>
__global__ __launch_bounds__(1024) void k_energy_stats(const T* __restrict__ e, int64_t n, double* __restrict__ out,
                                                       int finalize) {
  __shared__ double red[16];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) a += (double)e[i];
  const double nn = (double)n;
  const double m = block_sum_1024(a, red) / nn;
  double q = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double d = (double)e[i] - m;
    q += d * d;
  }
  q = block_sum_1024(q, red);
  if (threadIdx.x == 0) {
    out[0] = q;
    out[1] = nn * m;
    out[2] = nn * m * m;
    out[3] = nn;
    if (finalize) {
      out[4] = m;
      out[5] = q / nn;
    }
  }
}
__global__ void k_energy_stats_final(double* out) {
  if (threadIdx.x == 0) energy_stats_final(out);
}

// The energy-gradient weights of make_loss on one rank (Loss/loss.py:73-135 clipping, :206-208
// statistics, :256-265 tangent), one workgroup, every sum in double and in a fixed order:
//   m = mean(e) (the loss), variance = mean |e - m|^2;
//   clip (scale > 0, centre m; clip_from_median = False): tv = mean |x - c| per component,
//     clipped x = clamp(x, c - scale tv, c + scale tv); centre of the differences
//     dc = mean(clipped) (center_at_clipped) or m; diff = clipped - dc; aux = dc;
//   no clip: diff = e - m, aux = e (total_energy's clipped_energy, kept as written);
//   w_re = wscale Re diff,  w_im = wscale Im(diff + aux)  (the d log|psi| and d phase weights);
//   clipped_out = dc + diff (aux.clipped_energy; dc = m without clipping);
//   stats = [m_re, m_im, variance, dc_re, dc_im].
// e_im / w_im / clipped_im may be null (real local energies).  Replaces ~25 small torch launches
// per training step (and the host sync of the complex check) on the single-rank path.
template <typename T>
__global__ __launch_bounds__(1024) void k_loss_weights(const T* __restrict__ er, const T* __restrict__ ei, int64_t n,
                                                       double clip, int center_at_clipped, double wscale,
                                                       T* __restrict__ wr, T* __restrict__ wi, T* __restrict__ cr,
                                                       T* __restrict__ ci, double* __restrict__ stats) {
  __shared__ double red[16];
  const double nn = (double)n;
  const bool cplx = ei != nullptr;
  double a = 0.0, b = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    a += (double)er[i];
    if (cplx) b += (double)ei[i];
  }
  const double mr = block_sum_1024(a, red) / nn;
  const double mi = cplx ? block_sum_1024(b, red) / nn : 0.0;
  double q = 0.0, tr = 0.0, ti = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double dr = (double)er[i] - mr, di = cplx ? (double)ei[i] - mi : 0.0;
    q += dr * dr + di * di;
    tr += fabs(dr);
    ti += fabs(di);
  }
  const double var = block_sum_1024(q, red) / nn;
  const bool clipping = clip > 0.0;
  double lor = 0.0, hir = 0.0, loi = 0.0, hii = 0.0, dcr = mr, dci = mi;
  if (clipping) {
    const double tvr = block_sum_1024(tr, red) / nn;
    const double tvi = cplx ? block_sum_1024(ti, red) / nn : 0.0;
    lor = mr - clip * tvr;
    hir = mr + clip * tvr;
    loi = mi - clip * tvi;
    hii = mi + clip * tvi;
    if (center_at_clipped) {
      double sr = 0.0, si = 0.0;
      for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const double x = (double)er[i];
        sr += x < lor ? lor : (x > hir ? hir : x);
        if (cplx) {
          const double y = (double)ei[i];
          si += y < loi ? loi : (y > hii ? hii : y);
        }
      }
      dcr = block_sum_1024(sr, red) / nn;
      dci = cplx ? block_sum_1024(si, red) / nn : 0.0;
    }
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = (double)er[i], y = cplx ? (double)ei[i] : 0.0;
    double fr, fi, ar, ai;
    if (clipping) {
      const double xc = x < lor ? lor : (x > hir ? hir : x), yc = y < loi ? loi : (y > hii ? hii : y);
      fr = xc - dcr;
      fi = yc - dci;
      ar = dcr;
      ai = dci;
    } else {
      fr = x - mr;
      fi = y - mi;
      ar = x;
      ai = y;
    }
    wr[i] = (T)(wscale * fr);
    if (wi) wi[i] = (T)(wscale * (fi + ai));
    if (cr) cr[i] = (T)(dcr + fr);   // centre + diff (= e without clipping: dc = m)
    if (ci) ci[i] = (T)(dci + fi);
  }
  if (threadIdx.x == 0) {
    stats[0] = mr;
    stats[1] = mi;
    stats[2] = var;
    stats[3] = dcr;
    stats[4] = dci;
  }
}

// out[i] = grad[i] * taueff (limdrift, VMCmcstep.py:11-14 / drift_diffusion.py:9-12)
template <typename T>
__global__ __launch_bounds__(256) void k_scale_grad(const T* __restrict__ g, const double* __restrict__ taueff, int n,
                                                    T* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = g[i] * (T)taueff[0];
}

// DMC energy cut minima (S_matrix.py:21-22): jnp.min over the stacked [|e_est - eloc|, branchcut]
// array is ONE minimum over every walker (of every device: the reference stacks the pmapped
// [ndev, B] arrays) and the cut.  k_dmc_cut_part: part[2 blk], part[2 blk + 1] = this block's
// minima for eloc_old / eloc_new (the branch cut included); a minimum is exact in any order, so
// the consumers take the min over the DMC_NB block results directly.
// eest_b (nullable): per-walker e_est (the first block, main_dmc.py:115-116), else e_est.
template <typename T>
__global__ __launch_bounds__(256) void k_dmc_cut_part(int B, const T* __restrict__ eold, const T* __restrict__ enew,
                                                      const T* __restrict__ eest_b, double e_est, double branchcut,
                                                      double* __restrict__ part) {
  __shared__ double mo[256], mn[256];
  double a = branchcut, b = branchcut;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B; i += 256 * DMC_NB) {
    const double ee = eest_b ? (double)eest_b[i] : e_est;
    a = fmin(a, fabs(ee - (double)eold[i]));
    b = fmin(b, fabs(ee - (double)enew[i]));
  }
  mo[threadIdx.x] = a;
  mn[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      mo[threadIdx.x] = fmin(mo[threadIdx.x], mo[threadIdx.x + s]);
      mn[threadIdx.x] = fmin(mn[threadIdx.x], mn[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = mo[0];
    part[2 * blockIdx.x + 1] = mn[0];
  }
}
__global__ void k_dmc_cut_fin(const double* __restrict__ part, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double a = part[0], b = part[1];
  for (int k = 1; k < DMC_NB; ++k) {
    a = fmin(a, part[2 * k]);
    b = fmin(b, part[2 * k + 1]);
  }
  out[0] = a;
  out[1] = b;
}

// DMC weights (DMC/S_matrix.py:4-24, dmc.py:80-92), one thread per walker:
//   S = e_trial - e_est + e_cut / (1 + (v2 tau / N)^2), v2 = |grad_eff|^2 per walker,
//   e_cut = cut * sign(e_est - eloc_b), cut = the global minimum above: the caller's all-reduced
//   cuts[2] (multi-device run), or the min over k_dmc_cut_part's block minima of this batch (cpart),
//   w *= exp(tau tdamp (S_new + S_old) / 2).
// etr_b / eest_b (nullable): per-walker e_trial / e_est of the first DMC block.
template <typename T>
__global__ __launch_bounds__(256) void k_dmc_weights(int B, int N, const T* __restrict__ eold, const T* __restrict__ enew,
                                                     const T* __restrict__ gold, const T* __restrict__ gnew,
                                                     const double* __restrict__ tdamp, double tau,
                                                     const T* __restrict__ etr_b, const T* __restrict__ eest_b,
                                                     double e_trial, double e_est, const double* __restrict__ cuts,
                                                     const double* __restrict__ cpart, T* __restrict__ w) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  double cut_o, cut_n;
  if (cuts) {
    cut_o = cuts[0];
    cut_n = cuts[1];
  } else {
    cut_o = cpart[0];
    cut_n = cpart[1];
    for (int k = 1; k < DMC_NB; ++k) {
      cut_o = fmin(cut_o, cpart[2 * k]);
      cut_n = fmin(cut_n, cpart[2 * k + 1]);
    }
  }
  const double td = tdamp[2];   // [sum proposed, sum new, tdamp] of aiqmc_dmc_drift_diffusion
  double vo = 0.0, vn = 0.0;
  for (int k = 0; k < 3 * N; ++k) {
    const double x = (double)gold[(size_t)i * 3 * N + k], y = (double)gnew[(size_t)i * 3 * N + k];
    vo += x * x;
    vn += y * y;
  }
  const double ee = eest_b ? (double)eest_b[i] : e_est;
  const double et = etr_b ? (double)etr_b[i] : e_trial;
  const double co = ee - (double)eold[i], cn = ee - (double)enew[i];
  const double so = et - ee + cut_o * (double)((co > 0) - (co < 0)) / (1.0 + (vo * tau / N) * (vo * tau / N));
  const double sn = et - ee + cut_n * (double)((cn > 0) - (cn < 0)) / (1.0 + (vn * tau / N) * (vn * tau / N));
  w[i] = (T)(exp(tau * td * (0.5 * sn + 0.5 * so)) * (double)w[i]);
}

// Stochastic comb (DMC/branch.py:10-33), one block: cumulative weights in a fixed order, then
// newinds[j] = searchsorted_left(cumsum, (u wtot + j wtot / n) mod wtot); wout[0] = wtot / n.
// The cumulative sum is a blocked scan: thread t sums its contiguous chunk of ceil(n / 1024)
// weights, the 1024 chunk sums are scanned in a fixed tree (Hillis-Steele over LDS), and each
// thread re-walks its chunk from its prefix.  Deterministic; it equals the sequential sum up to
// fp64 rounding.  (A single thread carrying the running sum took 196 us at n = 4096 from global
// memory and 69 us through LDS.)  The searches read an LDS copy when the cumsum fits.
constexpr int COMB_LDS = 4096;
template <typename T>
__global__ __launch_bounds__(1024) void k_dmc_branch(int n, const T* __restrict__ w, double u, double* __restrict__ csum,
                                                     int32_t* __restrict__ newinds, T* __restrict__ wout) {
  __shared__ double sc[1024];
  __shared__ double cl[COMB_LDS];
  const int t = threadIdx.x;
  const int ch = (n + 1023) / 1024;
  const int i0 = t * ch < n ? t * ch : n, i1 = i0 + ch < n ? i0 + ch : n;
  double s = 0.0;
  for (int i = i0; i < i1; ++i) s += (double)w[i];
  sc[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {   // inclusive scan of the chunk sums
    const double v = t >= d ? sc[t - d] : 0.0;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  double a = t > 0 ? sc[t - 1] : 0.0;
  const bool lds = n <= COMB_LDS;
  for (int i = i0; i < i1; ++i) {
    a += (double)w[i];
    if (lds) cl[i] = a;
    else csum[i] = a;
  }
  __syncthreads();   // (block-scope fence: the global cumsum of the other threads is visible)
  const double* cp = lds ? cl : csum;
  const double wtot = cp[n - 1];
  for (int j = t; j < n; j += 1024) {
    const double tt = fmod(u * wtot + (double)j * (wtot / (double)n), wtot);
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cp[mid] < tt) lo = mid + 1;
      else hi = mid;
    }
    newinds[j] = lo;
  }
  if (t == 0) wout[0] = (T)(wtot / (double)n);
}

// ============================================================================ host side

static thread_local std::string g_err;
int aiqmc_fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
static int fail(int code, const std::string& m) { return aiqmc_fail(code, m); }
#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(AIQMC_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static bool shape_ops(int N, int A, ShapeOps* ops) {
#define AIQMC_CASE(n, a) \
  if (N == n && A == a) return aiqmc_shape_ops_##n##_##a(ops);
  AIQMC_SHAPE_LIST(AIQMC_CASE)
#undef AIQMC_CASE
  return false;
}

// DMC reduction scratch (2 * DMC_NB doubles), allocated on first use
static double* dmc_scratch(aiqmc_ctx* c) {
  if (!c->d_dscr && hipMalloc((void**)&c->d_dscr, 2 * DMC_NB * sizeof(double)) != hipSuccess) c->d_dscr = nullptr;
  return c->d_dscr;
}

static hipEvent_t ev_get(aiqmc_ctx* c) {
  if (!c->ev_free.empty()) {
    hipEvent_t e = c->ev_free.back();
    c->ev_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Launch `fn` on stream s; when profiling, bracket it with a pair of events in `slot`.
template <typename F>
static void timed(aiqmc_ctx* c, int slot, hipStream_t s, F&& fn) {
  if (!c->prof) {
    fn();
    return;
  }
  hipEvent_t a = ev_get(c), b = ev_get(c);
  if (!a || !b) {
    fn();
    return;
  }
  (void)hipEventRecord(a, s);
  fn();
  (void)hipEventRecord(b, s);
  c->ev_used[slot].push_back({a, b});
}

static void free_ws(aiqmc_ctx* c) {
  void* ps[] = {c->d_grad, c->d_lp, c->d_sq, c->d_lpn, c->d_gown, c->d_sqn, c->d_taueff, c->d_g1, c->d_g2, c->d_u,
                c->d_wc, c->d_ec};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  c->d_grad = c->d_lp = c->d_sq = c->d_lpn = c->d_gown = c->d_sqn = nullptr;
  c->d_g1 = c->d_g2 = c->d_u = nullptr;
  c->d_wc = c->d_ec = nullptr;
  c->d_taueff = nullptr;
  if (c->d_tacc) (void)hipFree(c->d_tacc);
  c->d_tacc = nullptr;
  c->tacc_n = 0;
  if (c->d_tpart) (void)hipFree(c->d_tpart);
  c->d_tpart = nullptr;
  c->tpart_n = 0;
  c->ws_B = 0;
  c->ws_bytes = 0;
}

static int ensure_ws(aiqmc_ctx* c, int B) {
  if (c->ws_B >= B) return 0;
  free_ws(c);
  const size_t s = c->dtype == AIQMC_F32 ? 4 : 8;
  const size_t N = (size_t)c->N;
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  size_t bytes[11] = {B * 3 * N * s, B * s, B * s, B * N * s, B * N * 3 * s, B * N * s,
                      B * N * 3 * s, B * N * 3 * s, B * N * s, B * (size_t)ops.wcache_n * s,
                      B * N * (size_t)ops.ecache_n * s};
  void** ptrs[11] = {&c->d_grad, &c->d_lp, &c->d_sq, &c->d_lpn, &c->d_gown, &c->d_sqn, &c->d_g1, &c->d_g2, &c->d_u,
                     &c->d_wc, &c->d_ec};
  int64_t tot = 0;
  for (int k = 0; k < 11; ++k) {
    HIPCHK(hipMalloc(ptrs[k], bytes[k]));
    tot += (int64_t)bytes[k];
  }
  HIPCHK(hipMalloc((void**)&c->d_taueff, 2 * sizeof(double)));

  c->ws_B = B;
  c->ws_bytes = tot + 16;
  return 0;
}

// per-proposal walker-cache scratch for the reuse-off diagnostics path (n configurations)
static int ensure_wcp(aiqmc_ctx* c, int64_t n, const ShapeOps& ops) {
  if (c->wcp_n >= n) return 0;
  if (c->d_wcp) (void)hipFree(c->d_wcp);
  c->d_wcp = nullptr;
  c->wcp_n = 0;
  HIPCHK(hipMalloc(&c->d_wcp, (size_t)n * ops.wcache_n * (c->dtype == AIQMC_F32 ? 4 : 8)));
  c->wcp_n = n;
  return 0;
}

static void free_ecp_ws(aiqmc_ctx* c) {
  void* ps[] = {c->d_ecp_rot, c->d_ecp_x, c->d_ecp_lq, c->d_ecp_pq, c->d_ecp_ec, c->d_ecp_el, c->d_ecp_lp0,
                c->d_ecp_ph0};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  c->d_ecp_rot = c->d_ecp_x = c->d_ecp_lq = c->d_ecp_pq = c->d_ecp_ec = nullptr;
  c->d_ecp_el = c->d_ecp_lp0 = c->d_ecp_ph0 = nullptr;
  c->ecp_B = 0;
  c->ecp_bytes = 0;
}

// ECP workspace for B walkers: B*N*A*50 quadrature configurations
static int ensure_ecp_ws(aiqmc_ctx* c, int B, const ShapeOps& ops) {
  if (c->ecp_B >= B) return 0;
  free_ecp_ws(c);
  const size_t s = c->dtype == AIQMC_F32 ? 4 : 8;
  const size_t nq = (size_t)B * c->N * c->A * ECP_NQ;
  size_t bytes[8] = {(size_t)B * 9 * s, nq * 3 * s, nq * s, nq * s, nq * (size_t)ops.ecache_n * s,
                     (size_t)B * s, (size_t)B * s, (size_t)B * s};
  void** ptrs[8] = {&c->d_ecp_rot, &c->d_ecp_x, &c->d_ecp_lq, &c->d_ecp_pq, &c->d_ecp_ec, &c->d_ecp_el,
                    &c->d_ecp_lp0, &c->d_ecp_ph0};
  int64_t tot = 0;
  for (int k = 0; k < 8; ++k) {
    HIPCHK(hipMalloc(ptrs[k], bytes[k]));
    tot += (int64_t)bytes[k];
  }
  c->ecp_B = B;
  c->ecp_bytes = tot;
  return 0;
}

// ============================================================================ C-ABI

extern "C" {

const char* aiqmc_last_error(void) { return g_err.c_str(); }

const char* aiqmc_supported_shapes(void) {
  static std::string s;
  if (s.empty()) {
#define AIQMC_NAME(n, a) s += (s.empty() ? "" : ",") + std::to_string(n) + ":" + std::to_string(a);
    AIQMC_SHAPE_LIST(AIQMC_NAME)
#undef AIQMC_NAME
  }
  return s.c_str();
}

int aiqmc_create(const aiqmc_cfg* cfg, aiqmc_ctx** out) {
  if (!cfg || !out) return fail(AIQMC_EINVAL, "null argument");
  *out = nullptr;
  const int N = cfg->nelectrons, A = cfg->natoms;
  if (N < 2 || N > 16) return fail(AIQMC_EUNSUPPORTED, "nelectrons must be in [2,16]");
  if (cfg->nspins[0] <= 0 || cfg->nspins[1] <= 0 || cfg->nspins[0] + cfg->nspins[1] != N)
    return fail(AIQMC_EUNSUPPORTED, "both spin channels must be occupied and sum to nelectrons");
  for (int l = 0; l < 3; ++l)
    if (cfg->hidden_dims[l][0] != NH || cfg->hidden_dims[l][1] != NH2 || cfg->hidden_dims_ynlm[l] != NYW)
      return fail(AIQMC_EUNSUPPORTED, "only the default hidden dims ((4,4),(4,4),(4,4)) / (6,6,6) are built");
  if (cfg->dtype != AIQMC_F32 && cfg->dtype != AIQMC_F64) return fail(AIQMC_EINVAL, "dtype");
  ShapeOps ops;
  if (!shape_ops(N, A, &ops))
    return fail(AIQMC_EUNSUPPORTED, "no kernel instantiation for (N,A)=(" + std::to_string(N) + "," +
                                        std::to_string(A) + "); supported: " + aiqmc_supported_shapes());
  if (cfg->n_parallel + cfg->n_antiparallel != N * (N - 1) / 2)
    return fail(AIQMC_EINVAL, "pair tables must cover all N(N-1)/2 pairs");
  aiqmc_ctx* c = new (std::nothrow) aiqmc_ctx();
  if (!c) return fail(AIQMC_EINVAL, "oom");
  c->N = N;
  c->A = A;
  c->nup = cfg->nspins[0];
  c->ndn = cfg->nspins[1];
  c->dtype = cfg->dtype;
  c->device = cfg->device;
  c->npar = cfg->n_parallel;
  c->nanti = cfg->n_antiparallel;
  c->atoms.assign(cfg->atoms, cfg->atoms + 3 * A);
  c->charges.assign(cfg->charges, cfg->charges + A);
  c->up.assign(cfg->spin_up_indices, cfg->spin_up_indices + c->nup);
  c->dn.assign(cfg->spin_down_indices, cfg->spin_down_indices + c->ndn);
  c->par.assign(cfg->parallel_indices, cfg->parallel_indices + 2 * c->npar);
  c->anti.assign(cfg->antiparallel_indices, cfg->antiparallel_indices + 2 * c->nanti);
  for (int v : c->up)
    if (v < 0 || v >= N) { delete c; return fail(AIQMC_EINVAL, "spin_up_indices out of range"); }
  for (int v : c->dn)
    if (v < 0 || v >= N) { delete c; return fail(AIQMC_EINVAL, "spin_down_indices out of range"); }
  for (int v : c->par)
    if (v < 0 || v >= N) { delete c; return fail(AIQMC_EINVAL, "parallel_indices out of range"); }
  for (int v : c->anti)
    if (v < 0 || v >= N) { delete c; return fail(AIQMC_EINVAL, "antiparallel_indices out of range"); }
  c->ncanon = ops.ncanon(c->npar, c->nanti);
  c->nkern = ops.nkern;
  c->nprm = ops.nprm;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) { delete c; return fail(AIQMC_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
  int rc = ops.set_lds();
  if (rc) { delete c; return rc; }
  if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->ncu <= 0)
    c->ncu = 256;
  const size_t s = c->dtype == AIQMC_F32 ? 4 : 8;
  e = hipMalloc(&c->d_prm, (size_t)c->nprm * s);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_rowsrc, 16 * sizeof(int));
  if (e != hipSuccess) {
    if (c->d_prm) (void)hipFree(c->d_prm);
    delete c;
    return fail(AIQMC_EHIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  int rows[16] = {0};
  for (int r = 0; r < c->nup; ++r) rows[r] = c->up[r];
  for (int r = 0; r < c->ndn; ++r) rows[c->nup + r] = c->dn[r];
  e = hipMemcpy(c->d_rowsrc, rows, sizeof(rows), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(c->d_prm);
    (void)hipFree(c->d_rowsrc);
    delete c;
    return fail(AIQMC_EHIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  *out = c;
  return AIQMC_OK;
}

int aiqmc_destroy(aiqmc_ctx* c) {
  if (!c) return AIQMC_OK;
  (void)hipSetDevice(c->device);
  free_ws(c);
  free_ecp_ws(c);
  if (c->d_tm_scr) (void)hipFree(c->d_tm_scr);
  if (c->d_dscr) (void)hipFree(c->d_dscr);
  if (c->d_ecp_tab) (void)hipFree(c->d_ecp_tab);
  void* pgp[] = {c->d_gmap, c->d_wnorm, c->d_pg, c->d_pgr, c->d_pk_op, c->d_pk_src, c->d_pk_cval};
  for (void* p : pgp)
    if (p) (void)hipFree(p);
  if (c->d_wcp) (void)hipFree(c->d_wcp);
  if (c->d_lc) (void)hipFree(c->d_lc);
  if (c->d_cx) (void)hipFree(c->d_cx);
  for (auto& v : c->ev_used)
    for (auto& p : v) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
  for (hipEvent_t e : c->ev_free) (void)hipEventDestroy(e);
  if (c->d_prm) (void)hipFree(c->d_prm);
  if (c->d_rowsrc) (void)hipFree(c->d_rowsrc);
  delete c;
  return AIQMC_OK;
}

int64_t aiqmc_param_count(const aiqmc_ctx* c) { return c ? c->ncanon : -1; }
int64_t aiqmc_workspace_bytes(const aiqmc_ctx* c) {
  return c ? c->ws_bytes + c->ecp_bytes + (int64_t)c->lc_B * c->lc_n * (c->dtype == AIQMC_F32 ? 4 : 8) : -1;
}

int aiqmc_set_params(aiqmc_ctx* c, const double* flat, int64_t n, void* stream) {
  if (!c || !flat) return fail(AIQMC_EINVAL, "null argument");
  if (n != c->ncanon)
    return fail(AIQMC_EINVAL, "expected " + std::to_string(c->ncanon) + " parameters, got " + std::to_string(n));
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  std::vector<double> lay;
  ops.pack(c, flat, lay);
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (c->dtype == AIQMC_F32) {
    std::vector<float> f(lay.begin(), lay.end());
    HIPCHK(hipMemcpyAsync(c->d_prm, f.data(), f.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
  } else {
    HIPCHK(hipMemcpyAsync(c->d_prm, lay.data(), lay.size() * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  // |W_y row| (the y coefficients are the last 6N canonical entries, nn.py:449-451), for the
  // canonical parameter gradient
  double wn[NYW];
  for (int m = 0; m < NYW; ++m) {
    double a = 0.0;
    for (int col = 0; col < c->N; ++col) {
      const double w = flat[n - NYW * c->N + m * c->N + col];
      a += w * w;
    }
    wn[m] = std::sqrt(a);
  }
  if (!c->d_wnorm) HIPCHK(hipMalloc((void**)&c->d_wnorm, NYW * sizeof(double)));
  HIPCHK(hipMemcpyAsync(c->d_wnorm, wn, sizeof(wn), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  c->params_set = true;
  return AIQMC_OK;
}

// Device repack of canonical parameters (fp64, device) into the kernel layout: the program is
// read off pack_params itself by two probes (flat_j = j + 1 and 2 (j + 1)): an entry equal in both is
// a constant of the system (atoms, charges, Jastrow cusps, V_nn), one that doubles is a copy of
// canonical j, and the W_y block is the row-normalised y coefficients (nn.py:449-451).  Per entry
// the arithmetic is pack_params' (double, same summation order for the row norms), so the kernel
// layout is bitwise the host upload's.
}  // extern "C"
template <typename T>
__global__ __launch_bounds__(256) void k_pack_params(const double* __restrict__ flat, const int* __restrict__ op,
                                                     const int* __restrict__ src, const double* __restrict__ cval,
                                                     int n, int wy_off, int wy_src0, int N, T* __restrict__ prm,
                                                     double* __restrict__ wnorm) {
  const int k = blockIdx.x * 256 + (int)threadIdx.x;
  if (k >= n) return;
  const int o = op[k];
  double v;
  if (o == 0) {
    v = cval[k];
  } else if (o == 1) {
    v = flat[src[k]];
  } else {
    const int m = (k - wy_off) / N;
    double a = 0.0;
    for (int col = 0; col < N; ++col) {
      // no fused multiply-add: the host's pack_params rounds the product and the sum apart
#pragma clang fp contract(off)
      const double w = flat[wy_src0 + m * N + col];
      a += w * w;
    }
    const double nrm = sqrt(a);
    v = flat[src[k]] / nrm;
    if (k - wy_off == m * N) wnorm[m] = nrm;
  }
  prm[k] = (T)v;
}

extern "C" {
static int build_pack_program(aiqmc_ctx* c, const ShapeOps& ops) {
  const int64_t n = c->ncanon;
  std::vector<double> fa(n), fb(n), la, lb;
  for (int64_t j = 0; j < n; ++j) {
    fa[j] = double(j + 1);
    fb[j] = 2.0 * double(j + 1);
  }
  ops.pack(c, fa.data(), la);
  ops.pack(c, fb.data(), lb);
  const int64_t nk = (int64_t)la.size();
  std::vector<int> op(nk, 0), src(nk, 0);
  std::vector<double> cval(nk, 0.0);
  const int wy_off = ops.wy_off, ny = NYW * c->N;
  const int64_t wy_src0 = n - ny;
  for (int64_t k = 0; k < nk; ++k) {
    if (k >= wy_off && k < wy_off + ny) {
      op[k] = 2;
      src[k] = (int)(wy_src0 + (k - wy_off));
    } else if (la[k] == lb[k]) {
      op[k] = 0;
      cval[k] = la[k];
    } else if (lb[k] == 2.0 * la[k] && la[k] >= 1.0 && la[k] <= double(n) && la[k] == std::floor(la[k])) {
      op[k] = 1;
      src[k] = (int)la[k] - 1;
    } else {
      return fail(AIQMC_EINVAL, "internal: kernel-layout entry " + std::to_string(k) + " is neither a copy nor a constant");
    }
  }
  HIPCHK(hipMalloc((void**)&c->d_pk_op, nk * sizeof(int)));
  HIPCHK(hipMalloc((void**)&c->d_pk_src, nk * sizeof(int)));
  HIPCHK(hipMalloc((void**)&c->d_pk_cval, nk * sizeof(double)));
  HIPCHK(hipMemcpy(c->d_pk_op, op.data(), nk * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_pk_src, src.data(), nk * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->d_pk_cval, cval.data(), nk * sizeof(double), hipMemcpyHostToDevice));
  return AIQMC_OK;
}

int aiqmc_set_params_device(aiqmc_ctx* c, const double* flat, int64_t n, void* stream) {
  if (!c || !flat) return fail(AIQMC_EINVAL, "null argument");
  if (n != c->ncanon)
    return fail(AIQMC_EINVAL, "expected " + std::to_string(c->ncanon) + " parameters, got " + std::to_string(n));
  HIPCHK(hipSetDevice(c->device));
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  if (!c->d_pk_op) {
    int rc = build_pack_program(c, ops);
    if (rc) return rc;
  }
  if (!c->d_wnorm) HIPCHK(hipMalloc((void**)&c->d_wnorm, NYW * sizeof(double)));
  const int nk = (int)ops.nprm;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((nk + 255) / 256), b(256);
  const int wy_src0 = (int)(n - NYW * c->N);
  if (c->dtype == AIQMC_F32)
    k_pack_params<float><<<g, b, 0, s>>>(flat, c->d_pk_op, c->d_pk_src, c->d_pk_cval, nk, ops.wy_off, wy_src0, c->N,
                                         (float*)c->d_prm, c->d_wnorm);
  else
    k_pack_params<double><<<g, b, 0, s>>>(flat, c->d_pk_op, c->d_pk_src, c->d_pk_cval, nk, ops.wy_off, wy_src0,
                                          c->N, (double*)c->d_prm, c->d_wnorm);
  HIPCHK(hipGetLastError());
  c->params_set = true;
  return AIQMC_OK;
}

static KArgs base_args(const aiqmc_ctx* c) {
  KArgs ka;
  std::memset(&ka, 0, sizeof(ka));
  ka.nup = c->nup;
  ka.rowsrc = c->d_rowsrc;
  ka.prm = c->d_prm;
  ka.one_wave = c->packed_walkers ? 0 : 1;
  return ka;
}

static int check_call(aiqmc_ctx* c, const void* pos, int B) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (!c->params_set) return fail(AIQMC_ESTATE, "aiqmc_set_params has not been called");
  if (B < 0) return fail(AIQMC_EINVAL, "negative batch");
  if (!pos && B > 0) return fail(AIQMC_EINVAL, "null positions");
  return 0;
}

int aiqmc_logpsi(aiqmc_ctx* c, const void* pos, int32_t B, void* logabs, void* phase, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = logabs;
  ka.phase = phase;
  rc = ensure_ws(c, B);
  if (rc) return rc;
  ka.wcache = c->d_wc;   // the kernel keeps its electron-local Jacobians there
  ops.walker(c->dtype, MODE_GRAD, ka, B, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_orbitals(aiqmc_ctx* c, const void* pos, int32_t B, void* orbitals, void* logabs, void* phase,
                   void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!orbitals) return fail(AIQMC_EINVAL, "null orbitals");
  HIPCHK(hipSetDevice(c->device));
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  rc = ensure_ws(c, B);
  if (rc) return rc;
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = logabs;
  ka.phase = phase;
  ka.value_only = 1;
  ka.orb = orbitals;
  ka.wcache = c->d_wc;
  ops.walker(c->dtype, MODE_GRAD, ka, B, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_logpsi_grad(aiqmc_ctx* c, const void* pos, int32_t B, void* logabs, void* grad, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!grad) return fail(AIQMC_EINVAL, "null grad");
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = logabs;
  ka.grad = grad;
  rc = ensure_ws(c, B);
  if (rc) return rc;
  ka.wcache = c->d_wc;
  ops.walker(c->dtype, MODE_GRAD, ka, B, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

// the local-energy launch pair for log|psi| (phase = 0: e_l = E_L) or theta = arg psi (phase = 1:
// e_l = the phase Laplacian, grad = grad theta)
static int local_energy_pass(aiqmc_ctx* c, const void* pos, int32_t B, void* e_l, void* logabs, void* grad, int phase,
                             void* stream) {
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  HIPCHK(hipSetDevice(c->device));
  if (c->lc_B < B) {
    if (c->d_lc) (void)hipFree(c->d_lc);
    c->d_lc = nullptr;
    c->lc_B = 0;
    HIPCHK(hipMalloc(&c->d_lc, (size_t)B * ops.lcache_n * (c->dtype == AIQMC_F32 ? 4 : 8)));
    c->lc_B = B;
    c->lc_n = ops.lcache_n;
  }
  // adjoint pass (values, h-stream adjoints, pair sums, B, Phi, Q_f) -> LapCache -> first-derivative pass
  KArgs k1 = base_args(c);
  k1.nconf = B;
  k1.pos = pos;
  k1.logabs = logabs;
  k1.lapcache = c->d_lc;
  KArgs k2 = base_args(c);
  k2.nconf = B;
  k2.pos = pos;
  k2.el = e_l;
  k2.grad = grad;
  k2.lapcache = c->d_lc;
  // waves per walker of the first-derivative pass: the fewest of 1, 2, 4 that give >= 2 waves per
  // SIMD (8 per CU); small per-GPU batches (strong scaling) split each walker over more waves
  int lw = c->lap_waves;
  if (lw <= 0) {
    const int64_t want = 8 * (int64_t)c->ncu;
    lw = (int64_t)B >= want ? 1 : ((int64_t)B * 2 >= want ? 2 : 4);
  }
  timed(c, 2, (hipStream_t)stream, [&] { ops.lap(c->dtype, k1, k2, B, lw, phase, (hipStream_t)stream); });
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_local_energy(aiqmc_ctx* c, const void* pos, int32_t B, void* e_l, void* logabs, void* grad,
                       void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!e_l) return fail(AIQMC_EINVAL, "null e_l");
  return local_energy_pass(c, pos, B, e_l, logabs, grad, 0, stream);
}

// complex-output scratch [B][6N+1]: grad log|psi|, grad theta, lap theta
static int ensure_cx(aiqmc_ctx* c, int B) {
  if (c->cx_B >= B) return AIQMC_OK;
  if (c->d_cx) (void)hipFree(c->d_cx);
  c->d_cx = nullptr;
  c->cx_B = 0;
  const size_t es = c->dtype == AIQMC_F32 ? 4 : 8;
  HIPCHK(hipMalloc(&c->d_cx, (size_t)B * (6 * c->N + 1) * es));
  c->cx_B = B;
  return AIQMC_OK;
}

int aiqmc_local_energy_complex(aiqmc_ctx* c, const void* pos, int32_t B, void* e_re, void* e_im, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!e_re || !e_im) return fail(AIQMC_EINVAL, "null e_re / e_im");
  HIPCHK(hipSetDevice(c->device));
  const int N = c->N;
  const size_t es = c->dtype == AIQMC_F32 ? 4 : 8;
  rc = ensure_cx(c, B);
  if (rc) return rc;
  char* gabs = (char*)c->d_cx;
  char* gph = gabs + (size_t)B * 3 * N * es;
  char* lph = gph + (size_t)B * 3 * N * es;
  rc = local_energy_pass(c, pos, B, e_re, nullptr, gabs, 0, stream);
  if (rc) return rc;
  rc = local_energy_pass(c, pos, B, lph, nullptr, gph, 1, stream);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((B + 255) / 256), b(256);
  if (c->dtype == AIQMC_F32)
    k_complex_el<float><<<g, b, 0, s>>>(B, 3 * N, (const float*)gabs, (const float*)gph, (const float*)lph,
                                         (float*)e_re, (float*)e_im);
  else
    k_complex_el<double><<<g, b, 0, s>>>(B, 3 * N, (const double*)gabs, (const double*)gph, (const double*)lph,
                                          (double*)e_re, (double*)e_im);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_debug_local_energy_forward(aiqmc_ctx* c, const void* pos, int32_t B, void* e_l, void* logabs, void* grad,
                                     void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!e_l) return fail(AIQMC_EINVAL, "null e_l");
  HIPCHK(hipSetDevice(c->device));
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.el = e_l;
  ka.logabs = logabs;
  ka.grad = grad;
  ops.walker(c->dtype, MODE_LAP, ka, B, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

// One drift-diffusion Metropolis sweep (VMCmcstep.py:28-111); step = Philox counter, st = index
// into host draws.  Launches: walker (+ the previous sweep's acceptance when *pending is set),
// limdrift, moved electron, proposals, limdrift, and -- unless `defer` -- the acceptance.  With
// `defer` the sweep's acceptance is left in *pending for the next sweep's walker launch (one
// launch and one inter-kernel gap fewer per sweep; same arithmetic, accept_one).
// dmc (optional, device doubles [3]): DMC drift-diffusion extras (DMC/drift_diffusion.py:15-22):
// dmc[0] = sum of the proposed coordinates, dmc[2] = tdamp = sum(x_new) / dmc[0]; never deferred.
// tacc (optional, fp32 mc_step): this sweep's zeroed pair of fused limdrift accumulators
// (walker_kernel.h TACC_SCALE); the two k_taueff launches are then skipped.
static int mc_sweep(aiqmc_ctx* c, const ShapeOps& ops, void* pos, int B, double tstep, int rng_mode, const void* gauss1,
                    const void* gauss2, const void* u, int st, uint64_t seed, uint64_t step, int32_t* accept_out,
                    double* dmc, hipStream_t s, AccArgs* pending = nullptr, bool defer = false,
                    unsigned long long* tacc = nullptr, unsigned long long* tpart = nullptr, bool pvok = false,
                    unsigned long long* zero_next = nullptr, int nzero = 0) {
  const int N = c->N;
  if (dmc) tacc = nullptr;
  if (dmc || tacc || c->dtype != AIQMC_F32) tpart = nullptr;
  const size_t es = c->dtype == AIQMC_F32 ? 4 : 8;
  double* dscr = dmc ? dmc_scratch(c) : nullptr;
  if (dmc && !dscr) return fail(AIQMC_EHIP, "hipMalloc: DMC scratch");
  const char* g1;
  const char* g2;
  const char* uu;
  if (rng_mode == AIQMC_RNG_HOST) {
    g1 = (const char*)gauss1 + (size_t)st * B * 3 * N * es;
    g2 = (const char*)gauss2 + (size_t)st * B * N * 3 * es;
    uu = (const char*)u + (size_t)st * B * N * es;
  } else {   // drawn by the walker launch below (k_draws' arithmetic, fused)
    g1 = (const char*)c->d_g1;
    g2 = (const char*)c->d_g2;
    uu = (const char*)c->d_u;
  }
  // (1) grad log|psi| at the walkers (VMCmcstep.py:41-53), after the previous sweep's moves
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = c->d_lp;
  ka.grad = c->d_grad;
  ka.sumsq = c->d_sq;
  ka.tacc = tacc;
  ka.wcache = c->d_wc;
  ka.pvok = (pvok && c->walker_fixed_gj) ? 1 : 0;
  ka.tstep = tstep;
  ka.seed = seed;
  ka.step = step;
  if (rng_mode != AIQMC_RNG_HOST) {
    ka.dg1 = c->d_g1;
    ka.dg2 = c->d_g2;
    ka.du = c->d_u;
  }
  if (pending && pending->lpn) {
    ka.acc = *pending;
    pending->lpn = nullptr;
  }
  timed(c, 1, s, [&] { ops.walker(c->dtype, MODE_GRAD, ka, B, s); });
  // (2) limdrift factor over the device batch (:60) -- fused: summed by the walker launch
  if (!tacc) {
    if (tpart)
      k_taueff_part<<<dim3(TPART), dim3(256), 0, s>>>((const float*)c->d_sq, B, tpart);
    else if (c->dtype == AIQMC_F32)
      k_taueff<float><<<dim3(1), dim3(1024), 0, s>>>((const float*)c->d_sq, B, tstep, c->d_taueff);
    else
      k_taueff<double><<<dim3(1), dim3(1024), 0, s>>>((const double*)c->d_sq, B, tstep, c->d_taueff);
  }
  // (3) single-electron proposals x^(i): value + gradient (:55-79, :95-97)
  KArgs kp = base_args(c);
  kp.nconf = B * N;
  kp.pos = pos;
  kp.proposal = 1;
  kp.pgrad = c->d_grad;
  kp.gauss1 = g1;
  kp.taueff = c->d_taueff;
  kp.tacc = tacc;
  kp.tpart = tpart;
  kp.tstep = tstep;
  kp.seed = seed;
  kp.step = step;
  kp.logabs = c->d_lpn;
  kp.gown = c->d_gown;
  kp.sumsq = c->d_sqn;
  kp.ablate = c->ablate;
  if (c->reuse) {
    // moved electron's local stage for all B*N proposals, then proposals from the walker caches
    kp.wcache = c->d_wc;
    kp.ecache = c->d_ec;
    ops.moved(c->dtype, kp, s);
  } else {
    kp.wcache = c->d_wcp;   // per-proposal scratch of the same layout
  }
  timed(c, 0, s, [&] { ops.walker(c->dtype, MODE_GRAD, kp, B * N, s); });
  // (4) limdrift factor of the proposal gradients over all B*N*3N entries (:80) -- fused:
  // summed by the proposal launch
  if (!tacc) {
    if (tpart)
      k_taueff_part<<<dim3(TPART), dim3(256), 0, s>>>((const float*)c->d_sqn, B * N, tpart + TPART_KIND);
    else if (c->dtype == AIQMC_F32)
      k_taueff<float><<<dim3(1), dim3(1024), 0, s>>>((const float*)c->d_sqn, B * N, tstep,
                         c->d_taueff + 1);
    else
      k_taueff<double><<<dim3(1), dim3(1024), 0, s>>>((const double*)c->d_sqn, B * N, tstep,
                         c->d_taueff + 1);
  }
  if (dmc) {
    if (c->dtype == AIQMC_F32)
      k_dmc_sum_part<float><<<dim3(DMC_NB), dim3(256), 0, s>>>((const float*)pos, (const float*)c->d_grad,
                                                               (const float*)g1, c->d_taueff, tstep, B * 3 * N, dscr);
    else
      k_dmc_sum_part<double><<<dim3(DMC_NB), dim3(256), 0, s>>>((const double*)pos, (const double*)c->d_grad,
                                                                (const double*)g1, c->d_taueff, tstep, B * 3 * N, dscr);
    k_dmc_sum_fin<<<dim3(1), dim3(64), 0, s>>>(dscr, 1, dmc);
  }
  // (5) acceptance and move (:83-106)
  AccArgs a;
  a.grad = c->d_grad;
  a.lp = c->d_lp;
  a.lpn = c->d_lpn;
  a.gown = c->d_gown;
  a.gauss1 = g1;
  a.gauss2 = g2;
  a.u = uu;
  a.taueff = c->d_taueff;
  a.tacc = tacc;
  a.tpart = tpart;
  a.tstep = tstep;
  a.count = accept_out;
  if (defer && pending && !dmc) {
    *pending = a;
    return 0;
  }
  a.zero = zero_next;
  a.nzero = nzero;
  ops.accept(c->dtype, pos, a, B, s);
  if (dmc) {
    if (c->dtype == AIQMC_F32)
      k_dmc_sum_part<float><<<dim3(DMC_NB), dim3(256), 0, s>>>((const float*)pos, nullptr, nullptr, nullptr, tstep,
                                                               B * 3 * N, dscr);
    else
      k_dmc_sum_part<double><<<dim3(DMC_NB), dim3(256), 0, s>>>((const double*)pos, nullptr, nullptr, nullptr, tstep,
                                                                B * 3 * N, dscr);
    k_dmc_sum_fin<<<dim3(1), dim3(64), 0, s>>>(dscr, 0, dmc);
  }
  return 0;
}

int aiqmc_mc_step(aiqmc_ctx* c, void* pos, int32_t B, int32_t nsteps, double tstep, int32_t rng_mode,
                  const void* gauss1, const void* gauss2, const void* u, uint64_t seed, uint64_t offset,
                  int32_t* accept_out, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (nsteps < 0) return fail(AIQMC_EINVAL, "negative nsteps");
  if (!(tstep > 0.0)) return fail(AIQMC_EINVAL, "tstep must be > 0");
  if (rng_mode == AIQMC_RNG_HOST && B > 0 && (!gauss1 || !gauss2 || !u))
    return fail(AIQMC_EINVAL, "AIQMC_RNG_HOST needs gauss1, gauss2 and u");
  if (rng_mode != AIQMC_RNG_HOST && rng_mode != AIQMC_RNG_PHILOX) return fail(AIQMC_EINVAL, "rng_mode");
  if (B == 0 || nsteps == 0) return AIQMC_OK;
  HIPCHK(hipSetDevice(c->device));
  rc = ensure_ws(c, B);
  if (rc) return rc;
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  if (!c->reuse) {
    rc = ensure_wcp(c, (int64_t)B * c->N, ops);
    if (rc) return rc;
  }
  hipStream_t s = (hipStream_t)stream;
  // fp32: the limdrift sums of every sweep accumulate in integer accumulators (walker_kernel.h;
  // one set per sweep, zeroed once here) instead of two reduction launches per sweep.  N2, ms per
  // VMC iteration, launches vs fused: round 3 (1024 slots) 512 walkers 1.040 vs 1.000, 1024
  // walkers 1.399 vs 1.377, 4096 walkers 3.53 vs 3.56 (the consumers' wave-wide read of the 1024
  // slots cost more than the launches); round 4 with 256 slots, 4096 walkers 3.026-3.030 vs
  // 2.993-3.000.
  unsigned long long* tacc = nullptr;
  // (integer sums need fewer than TACC_MAX_CONF configurations per reduction, walker_kernel.h)
  const bool int_sums = (int64_t)B * c->N < TACC_MAX_CONF;
  if (int_sums && c->fuse_reduce && c->dtype == AIQMC_F32 && (c->fuse_reduce > 1 || B <= FUSE_REDUCE_MAX_B)) {
    // two banks of per-sweep accumulator sets: a call sums into bank p, and its last k_accept
    // zeroes bank 1 - p for the next call (round 5: no memset launch per call);
    // a bank not known to be clean (new allocation, an earlier call that stopped early) is
    // memset here
    if (c->tacc_n < nsteps) {
      if (c->d_tacc) (void)hipFree(c->d_tacc);
      c->d_tacc = nullptr;
      c->tacc_n = 0;
      c->tacc_clean[0] = c->tacc_clean[1] = false;
      HIPCHK(hipMalloc((void**)&c->d_tacc, (size_t)2 * 2 * TACC_STRIDE * nsteps * sizeof(unsigned long long)));
      c->tacc_n = nsteps;
    }
    const size_t bank_words = (size_t)2 * TACC_STRIDE * c->tacc_n;
    tacc = c->d_tacc + bank_words * c->tacc_bank;
    if (!c->tacc_clean[c->tacc_bank]) HIPCHK(hipMemsetAsync(tacc, 0, (size_t)2 * TACC_STRIDE * nsteps * sizeof(unsigned long long), s));
    c->tacc_clean[c->tacc_bank] = false;   // in use from here on
  }
  // unfused fp32 sweeps: per-sweep partial sums of the limdrift reductions (k_taueff_part), kept
  // until the next sweep's walker launch has read them (fused acceptance)
  unsigned long long* tpart = nullptr;
  if (int_sums && !tacc && c->dtype == AIQMC_F32 && c->wide_reduce) {
    if (c->tpart_n < nsteps) {
      if (c->d_tpart) (void)hipFree(c->d_tpart);
      c->d_tpart = nullptr;
      c->tpart_n = 0;
      HIPCHK(hipMalloc((void**)&c->d_tpart, (size_t)2 * TPART_KIND * nsteps * sizeof(unsigned long long)));
      c->tpart_n = nsteps;
    }
    tpart = c->d_tpart;
  }
  AccArgs pending{};
  const int other = 1 - c->tacc_bank;
  unsigned long long* zero_next = tacc ? c->d_tacc + (size_t)2 * TACC_STRIDE * c->tacc_n * other : nullptr;
  const int nzero = tacc ? 2 * TACC_STRIDE * c->tacc_n : 0;
  for (int st = 0; st < nsteps; ++st) {
    const bool last = st + 1 == nsteps;
    rc = mc_sweep(c, ops, pos, B, tstep, rng_mode, gauss1, gauss2, u, st, seed, offset + (uint64_t)st, accept_out,
                  nullptr, s, &pending, c->fuse_accept && !last, tacc ? tacc + 2 * TACC_STRIDE * st : nullptr,
                  tpart ? tpart + 2 * TPART_KIND * st : nullptr, st > 0, last ? zero_next : nullptr,
                  last ? nzero : 0);
    if (rc) return rc;
  }
  HIPCHK(hipGetLastError());
  if (tacc) {   // the last k_accept has zeroed the other bank: the next call uses it as it is
    c->tacc_clean[other] = true;
    c->tacc_bank = other;
  }
  return AIQMC_OK;
}

}  // extern "C"

// d log|psi| / d theta (phase = false) or d phase / d theta (phase = true), per walker or
// weighted sum, in canonical order.  vals: log|psi| or phase at the walkers (optional).
static int param_grad(aiqmc_ctx* c, const void* pos, int32_t B, const void* weights, void* out, void* vals,
                      bool phase, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!out) return fail(AIQMC_EINVAL, "null out");
  HIPCHK(hipSetDevice(c->device));
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  const size_t es = c->dtype == AIQMC_F32 ? 4 : 8;
  if (!c->d_gmap) {
    std::vector<int> map;
    ops.gmap(c, map);
    if ((int64_t)map.size() != c->ncanon) return fail(AIQMC_EINVAL, "internal: gradient map size");
    HIPCHK(hipMalloc((void**)&c->d_gmap, map.size() * sizeof(int)));
    HIPCHK(hipMemcpy(c->d_gmap, map.data(), map.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  if (c->pg_B < B) {
    if (c->d_pg) (void)hipFree(c->d_pg);
    if (c->d_pgr) (void)hipFree(c->d_pgr);
    c->d_pg = c->d_pgr = nullptr;
    c->pg_B = 0;
    HIPCHK(hipMalloc(&c->d_pg, (size_t)B * c->nkern * es));
    // row 0: the weighted sum; rows 1..: k_grad_partial's per-chunk sums
    HIPCHK(hipMalloc(&c->d_pgr, (size_t)(1 + (B + GR_CH - 1) / GR_CH) * c->nkern * es));
    c->pg_B = B;
  }
  hipStream_t s = (hipStream_t)stream;
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.grad = c->d_pg;
  ka.logabs = phase ? nullptr : vals;
  ka.phase = phase ? vals : nullptr;
  ka.phase_grad = phase ? 1 : 0;
  rc = ops.pgrad(c->dtype, ka, B, s);
  if (rc) return rc;
  const int nk = (int)c->nkern, nc = (int)c->ncanon;
  const void* G = c->d_pg;
  int rows = B;
  if (weights) {
    const int nch = (B + GR_CH - 1) / GR_CH;
    const dim3 gp((nk + 63) / 64, nch), gf((nk + 255) / 256);
    if (c->dtype == AIQMC_F32) {
      float* pr = (float*)c->d_pgr;
      k_grad_partial<float><<<gp, dim3(256), 0, s>>>((const float*)c->d_pg, (const float*)weights, B, nk, pr + nk);
      k_grad_final<float><<<gf, dim3(256), 0, s>>>(pr + nk, nch, nk, pr);
    } else {
      double* pr = (double*)c->d_pgr;
      k_grad_partial<double><<<gp, dim3(256), 0, s>>>((const double*)c->d_pg, (const double*)weights, B, nk, pr + nk);
      k_grad_final<double><<<gf, dim3(256), 0, s>>>(pr + nk, nch, nk, pr);
    }
    G = c->d_pgr;
    rows = 1;
  }
  const size_t nt = (size_t)rows * nc;
  const int nb = (int)((nt + 255) / 256);
  if (c->dtype == AIQMC_F32)
    k_grad_canon<float><<<dim3(nb), dim3(256), 0, s>>>((const float*)G, nk, c->d_gmap, nc,
                                                        (const float*)c->d_prm + ops.wy_off, ops.wy_off, c->d_wnorm,
                                                        c->N, rows, (float*)out);
  else
    k_grad_canon<double><<<dim3(nb), dim3(256), 0, s>>>((const double*)G, nk, c->d_gmap, nc,
                                                         (const double*)c->d_prm + ops.wy_off, ops.wy_off,
                                                         c->d_wnorm, c->N, rows, (double*)out);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

extern "C" {

int aiqmc_logpsi_param_grad(aiqmc_ctx* c, const void* pos, int32_t B, const void* weights, void* out,
                            void* logabs, void* stream) {
  return param_grad(c, pos, B, weights, out, logabs, false, stream);
}

int aiqmc_phase_param_grad(aiqmc_ctx* c, const void* pos, int32_t B, const void* weights, void* out, void* phase,
                           void* stream) {
  return param_grad(c, pos, B, weights, out, phase, true, stream);
}

int aiqmc_set_ecp(aiqmc_ctx* c, const aiqmc_ecp* e) {
  if (!c || !e) return fail(AIQMC_EINVAL, "null argument");
  if (e->list_l < 0 || e->list_l > 3) return fail(AIQMC_EUNSUPPORTED, "list_l must be in [0,3] (P_l, pseudopotential.py:250-269)");
  if (e->n_local < 0 || e->n_nonlocal < 0) return fail(AIQMC_EINVAL, "negative table size");
  if ((e->n_local && (!e->rn_local || !e->local_coes || !e->local_exps)) ||
      (e->n_nonlocal && (!e->rn_non_local || !e->non_local_coes || !e->non_local_exps)))
    return fail(AIQMC_EINVAL, "null ECP table");
  const int A = c->A, KL = e->n_local, KN = e->n_nonlocal, L = e->list_l + 1;
  // device table: atoms [A][3], charges [A], then per atom KL local and L*KN nonlocal (n, c, alpha)
  std::vector<double> tab(4 * A + (size_t)A * 3 * (KL + L * KN));
  for (int a = 0; a < A; ++a) {
    for (int d = 0; d < 3; ++d) tab[a * 3 + d] = c->atoms[a * 3 + d];
    tab[3 * A + a] = c->charges[a];
    double* t = tab.data() + 4 * A + (size_t)a * 3 * (KL + L * KN);
    for (int k = 0; k < KL; ++k) {
      t[3 * k] = e->rn_local[a * KL + k];
      t[3 * k + 1] = e->local_coes[a * KL + k];
      t[3 * k + 2] = e->local_exps[a * KL + k];
    }
    t += 3 * KL;
    for (int k = 0; k < L * KN; ++k) {
      t[3 * k] = e->rn_non_local[(size_t)a * L * KN + k];
      t[3 * k + 1] = e->non_local_coes[(size_t)a * L * KN + k];
      t[3 * k + 2] = e->non_local_exps[(size_t)a * L * KN + k];
    }
  }
  HIPCHK(hipSetDevice(c->device));
  if (c->d_ecp_tab) (void)hipFree(c->d_ecp_tab);
  c->d_ecp_tab = nullptr;
  c->ecp_set = false;
  HIPCHK(hipMalloc((void**)&c->d_ecp_tab, tab.size() * sizeof(double)));
  HIPCHK(hipMemcpy(c->d_ecp_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
  c->ecp_KL = KL;
  c->ecp_KN = KN;
  c->ecp_L = L;
  c->ecp_nl_zero = true;
  for (size_t k = 0; k < (size_t)A * L * KN; ++k)
    if (e->non_local_coes[k] != 0.0) c->ecp_nl_zero = false;
  c->ecp_set = true;
  return AIQMC_OK;
}

}  // extern "C"

// Steps shared by the pp local energy and the T-moves (pseudopotential.py:272-318): per-walker
// rotations (Philox draws or the caller's), the N*A*50 moved-electron positions, log psi at the
// walkers (walker launch, which also fills the walker cache) and at every quadrature
// configuration (value-only proposal launch through the cache).
static int ecp_quadrature(aiqmc_ctx* c, const void* pos, int B, int rng_mode, const void* rot, uint64_t seed,
                          uint64_t offset, void* logabs_q, void* phase_q, EcpArgs& ea, hipStream_t s) {
  const int64_t M = (int64_t)c->N * c->A * ECP_NQ;
  if ((int64_t)B * M > INT32_MAX) return fail(AIQMC_EINVAL, "too many quadrature configurations for one call");
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  int rc = ensure_ws(c, B);
  if (rc) return rc;
  if (!c->reuse) {
    rc = ensure_wcp(c, (int64_t)B * M, ops);
    if (rc) return rc;
  }
  const int nq = (int)(B * M);
  void* lq = logabs_q ? logabs_q : c->d_ecp_lq;
  void* pq = phase_q ? phase_q : c->d_ecp_pq;
  std::memset(&ea, 0, sizeof(ea));
  ea.B = B;
  ea.N = c->N;
  ea.A = c->A;
  ea.KL = c->ecp_KL;
  ea.KN = c->ecp_KN;
  ea.L = c->ecp_L;
  ea.tab = c->d_ecp_tab;
  ea.pos = pos;
  ea.rot = rng_mode == AIQMC_RNG_HOST ? rot : c->d_ecp_rot;
  ea.lp0 = c->d_ecp_lp0;
  ea.ph0 = c->d_ecp_ph0;
  ea.lpq = lq;
  ea.phq = pq;
  ea.xnew = c->d_ecp_x;
  ea.seed = seed;
  ea.step = offset;
  const bool f32 = c->dtype == AIQMC_F32;
  if (rng_mode == AIQMC_RNG_PHILOX) {
    if (f32) k_ecp_rot<float><<<dim3((B + 255) / 256), dim3(256), 0, s>>>(ea);
    else k_ecp_rot<double><<<dim3((B + 255) / 256), dim3(256), 0, s>>>(ea);
  }
  if (f32) k_ecp_points<float><<<dim3((nq + 255) / 256), dim3(256), 0, s>>>(ea);
  else k_ecp_points<double><<<dim3((nq + 255) / 256), dim3(256), 0, s>>>(ea);
  // walker launch: log psi at the walkers + the walker cache
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = c->d_ecp_lp0;
  ka.phase = c->d_ecp_ph0;
  ka.wcache = c->d_wc;
  ops.walker(c->dtype, MODE_GRAD, ka, B, s);
  // quadrature configurations: one moved electron each, value only
  KArgs kp = base_args(c);
  kp.nconf = nq;
  kp.pos = pos;
  kp.proposal = 1;
  kp.mper = (int)M;
  kp.mdiv = c->A * ECP_NQ;
  kp.xnew = c->d_ecp_x;
  kp.value_only = 1;
  kp.logabs = lq;
  kp.phase = pq;
  if (c->reuse) {
    kp.wcache = c->d_wc;
    kp.ecache = c->d_ecp_ec;
    ops.moved(c->dtype, kp, s);
  } else {
    kp.wcache = c->d_wcp;
  }
  timed(c, 3, s, [&] { ops.walker(c->dtype, MODE_GRAD, kp, nq, s); });
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

extern "C" {

static int local_energy_ecp_impl(aiqmc_ctx* c, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                                 uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* logabs_q,
                                 void* phase_q, bool cplx, void* stream);

int aiqmc_local_energy_ecp(aiqmc_ctx* c, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                           uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* logabs_q, void* phase_q,
                           void* stream) {
  return local_energy_ecp_impl(c, pos, B, rng_mode, rot, seed, offset, e_re, e_im, logabs_q, phase_q, false, stream);
}

int aiqmc_local_energy_ecp_complex(aiqmc_ctx* c, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                                   uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* stream) {
  return local_energy_ecp_impl(c, pos, B, rng_mode, rot, seed, offset, e_re, e_im, nullptr, nullptr, true, stream);
}

static int local_energy_ecp_impl(aiqmc_ctx* c, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                                 uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* logabs_q,
                                 void* phase_q, bool cplx, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (!c->ecp_set) return fail(AIQMC_ESTATE, "aiqmc_set_ecp has not been called");
  if (rng_mode == AIQMC_RNG_HOST && B > 0 && !rot) return fail(AIQMC_EINVAL, "AIQMC_RNG_HOST needs rot");
  if (rng_mode != AIQMC_RNG_HOST && rng_mode != AIQMC_RNG_PHILOX) return fail(AIQMC_EINVAL, "rng_mode");
  if (B == 0) return AIQMC_OK;
  if (!e_re || !e_im) return fail(AIQMC_EINVAL, "null e_re / e_im");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  // (1) all-electron local energy V + KE (walker_lap.h)
  {
    ShapeOps ops0;
    shape_ops(c->N, c->A, &ops0);
    rc = ensure_ecp_ws(c, B, ops0);
    if (rc) return rc;
  }
  const size_t es = c->dtype == AIQMC_F32 ? 4 : 8;
  char* gabs = nullptr;
  if (cplx) {
    // complex_output=True (pphamiltonian.py:84-104 = hamiltonian.py:110-130): the all-electron
    // pass also leaves grad log|psi|, and the phase pass gives grad theta and lap theta
    rc = ensure_cx(c, B);
    if (rc) return rc;
    gabs = (char*)c->d_cx;
    rc = local_energy_pass(c, pos, B, c->d_ecp_el, nullptr, gabs, 0, stream);
    if (rc) return rc;
    rc = local_energy_pass(c, pos, B, gabs + (size_t)2 * B * 3 * c->N * es, nullptr, gabs + (size_t)B * 3 * c->N * es,
                           1, stream);
  } else {
    rc = aiqmc_local_energy(c, pos, B, c->d_ecp_el, nullptr, nullptr, stream);
  }
  if (rc) return rc;
  // (2)-(4) rotations, quadrature positions, log psi at the walkers and the quadrature points --
  // skipped when every nonlocal coefficient is 0 (all-electron tables, "Ne + DMC"): each
  // quadrature term is 0 times a finite log-ratio (E4), so only the local part remains
  EcpArgs ea;
  if (c->ecp_nl_zero && !logabs_q && !phase_q) {
    std::memset(&ea, 0, sizeof(ea));
    ea.B = B;
    ea.N = c->N;
    ea.A = c->A;
    ea.KL = c->ecp_KL;
    ea.KN = c->ecp_KN;
    ea.L = c->ecp_L;
    ea.tab = c->d_ecp_tab;
    ea.pos = pos;
    ea.skip_nl = 1;
  } else {
    rc = ecp_quadrature(c, pos, B, rng_mode, rot, seed, offset, logabs_q, phase_q, ea, s);
    if (rc) return rc;
  }
  ea.eall = c->d_ecp_el;
  ea.e_re = e_re;
  ea.e_im = e_im;
  // (5) local pp part + nonlocal quadrature sum
  if (c->dtype == AIQMC_F32) k_ecp_energy<float><<<dim3(B), dim3(64), 0, s>>>(ea);
  else k_ecp_energy<double><<<dim3(B), dim3(64), 0, s>>>(ea);
  if (cplx) {   // + 1/2 |grad theta|^2 - i (lap theta / 2 + grad log|psi| . grad theta)
    const char* gph = gabs + (size_t)B * 3 * c->N * es;
    const char* lph = gph + (size_t)B * 3 * c->N * es;
    const dim3 g((B + 255) / 256), b(256);
    if (c->dtype == AIQMC_F32)
      k_complex_el<float, true><<<g, b, 0, s>>>(B, 3 * c->N, (const float*)gabs, (const float*)gph,
                                                 (const float*)lph, (float*)e_re, (float*)e_im);
    else
      k_complex_el<double, true><<<g, b, 0, s>>>(B, 3 * c->N, (const double*)gabs, (const double*)gph,
                                                  (const double*)lph, (double*)e_re, (double*)e_im);
  }
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_dmc_tmoves(aiqmc_ctx* c, void* pos, int32_t B, double tstep, int32_t rng_mode, const void* rot,
                     const void* u_sel, const void* u_acc, uint64_t seed, uint64_t offset, void* acceptance,
                     void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (!c->ecp_set) return fail(AIQMC_ESTATE, "aiqmc_set_ecp has not been called");
  if (!(tstep > 0.0)) return fail(AIQMC_EINVAL, "tstep must be > 0");
  if (rng_mode == AIQMC_RNG_HOST && B > 0 && (!rot || !u_sel || !u_acc))
    return fail(AIQMC_EINVAL, "AIQMC_RNG_HOST needs rot, u_sel and u_acc");
  if (rng_mode != AIQMC_RNG_HOST && rng_mode != AIQMC_RNG_PHILOX) return fail(AIQMC_EINVAL, "rng_mode");
  if (B == 0) return AIQMC_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (c->ecp_nl_zero) {   // no T-move amplitude: nothing moves, acceptance exactly 1 (k_tmove_none)
    if (acceptance) {
      const int n = B * c->N;
      if (c->dtype == AIQMC_F32) k_tmove_none<float><<<dim3((n + 255) / 256), dim3(256), 0, s>>>((float*)acceptance, n);
      else k_tmove_none<double><<<dim3((n + 255) / 256), dim3(256), 0, s>>>((double*)acceptance, n);
      HIPCHK(hipGetLastError());
    }
    return AIQMC_OK;
  }
  {
    ShapeOps ops0;
    shape_ops(c->N, c->A, &ops0);
    rc = ensure_ecp_ws(c, B, ops0);
    if (rc) return rc;
  }
  if (!c->d_tm_scr || c->tm_B < B) {
    if (c->d_tm_scr) HIPCHK(hipFree(c->d_tm_scr));
    c->d_tm_scr = nullptr;
    c->tm_B = 0;
    HIPCHK(hipMalloc(&c->d_tm_scr, (size_t)B * c->N * c->A * ECP_NQ * 4 * sizeof(double)));
    c->tm_B = B;
  }
  EcpArgs ea;
  rc = ecp_quadrature(c, pos, B, rng_mode, rot, seed, offset, nullptr, nullptr, ea, s);
  if (rc) return rc;
  ea.tstep = tstep;
  ea.usel = rng_mode == AIQMC_RNG_HOST ? u_sel : nullptr;
  ea.uacc = rng_mode == AIQMC_RNG_HOST ? u_acc : nullptr;
  ea.acc = acceptance;
  ea.pos_out = pos;
  ea.scr = c->d_tm_scr;
  if (c->dtype == AIQMC_F32) k_tmove<float><<<dim3(B), dim3(64), 0, s>>>(ea);
  else k_tmove<double><<<dim3(B), dim3(64), 0, s>>>(ea);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_dmc_drift_diffusion(aiqmc_ctx* c, void* pos, int32_t B, double tstep, int32_t rng_mode, const void* gauss1,
                              const void* gauss2, const void* u, uint64_t seed, uint64_t offset, void* grad_eff_old,
                              void* grad_new_eff, double* tdamp, void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (!(tstep > 0.0)) return fail(AIQMC_EINVAL, "tstep must be > 0");
  if (rng_mode == AIQMC_RNG_HOST && B > 0 && (!gauss1 || !gauss2 || !u))
    return fail(AIQMC_EINVAL, "AIQMC_RNG_HOST needs gauss1, gauss2 and u");
  if (rng_mode != AIQMC_RNG_HOST && rng_mode != AIQMC_RNG_PHILOX) return fail(AIQMC_EINVAL, "rng_mode");
  if (B == 0) return AIQMC_OK;
  if (!grad_eff_old || !grad_new_eff || !tdamp) return fail(AIQMC_EINVAL, "null output");
  HIPCHK(hipSetDevice(c->device));
  rc = ensure_ws(c, B);
  if (rc) return rc;
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  if (!c->reuse) {
    rc = ensure_wcp(c, (int64_t)B * c->N, ops);
    if (rc) return rc;
  }
  hipStream_t s = (hipStream_t)stream;
  const int n = B * 3 * c->N;
  const int nb = (n + 255) / 256;
  rc = mc_sweep(c, ops, pos, B, tstep, rng_mode, gauss1, gauss2, u, 0, seed, offset, nullptr, tdamp, s);
  if (rc) return rc;
  // grad_eff_old: limdrift of the walker gradients of this sweep (drift_diffusion.py:60-61)
  if (c->dtype == AIQMC_F32)
    k_scale_grad<float><<<dim3(nb), dim3(256), 0, s>>>((const float*)c->d_grad, c->d_taueff, n, (float*)grad_eff_old);
  else
    k_scale_grad<double><<<dim3(nb), dim3(256), 0, s>>>((const double*)c->d_grad, c->d_taueff, n,
                                                         (double*)grad_eff_old);
  // grad_new_eff_s: limdrift of the gradients at the moved walkers (:103-104)
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.grad = grad_new_eff;
  ka.sumsq = c->d_sq;
  ka.wcache = c->d_wc;
  ops.walker(c->dtype, MODE_GRAD, ka, B, s);
  if (c->dtype == AIQMC_F32) {
    k_taueff<float><<<dim3(1), dim3(1024), 0, s>>>((const float*)c->d_sq, B, tstep, c->d_taueff + 1);
    k_scale_grad<float><<<dim3(nb), dim3(256), 0, s>>>((const float*)grad_new_eff, c->d_taueff + 1, n,
                                                        (float*)grad_new_eff);
  } else {
    k_taueff<double><<<dim3(1), dim3(1024), 0, s>>>((const double*)c->d_sq, B, tstep, c->d_taueff + 1);
    k_scale_grad<double><<<dim3(nb), dim3(256), 0, s>>>((const double*)grad_new_eff, c->d_taueff + 1, n,
                                                         (double*)grad_new_eff);
  }
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_dmc_weights_ex(aiqmc_ctx* c, int32_t B, const void* eloc_old, const void* eloc_new,
                         const void* grad_eff_old, const void* grad_new_eff, const double* tdamp, double tstep,
                         const void* e_trial_b, const void* e_est_b, double e_trial, double e_est, double branchcut,
                         const double* cut_minima, void* weights_inout, void* stream) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (B < 0) return fail(AIQMC_EINVAL, "negative batch");
  if (B == 0) return AIQMC_OK;
  if (!eloc_old || !eloc_new || !grad_eff_old || !grad_new_eff || !tdamp || !weights_inout)
    return fail(AIQMC_EINVAL, "null argument");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const double* cpart = nullptr;
  if (!cut_minima) {   // this batch's minima (single device)
    double* d = dmc_scratch(c);
    if (!d) return fail(AIQMC_EHIP, "hipMalloc: DMC scratch");
    if (c->dtype == AIQMC_F32)
      k_dmc_cut_part<float><<<dim3(DMC_NB), dim3(256), 0, s>>>(B, (const float*)eloc_old, (const float*)eloc_new,
                                                               (const float*)e_est_b, e_est, branchcut, d);
    else
      k_dmc_cut_part<double><<<dim3(DMC_NB), dim3(256), 0, s>>>(B, (const double*)eloc_old, (const double*)eloc_new,
                                                                (const double*)e_est_b, e_est, branchcut, d);
    cpart = d;
  }
  const dim3 gw((B + 255) / 256);
  if (c->dtype == AIQMC_F32)
    k_dmc_weights<float><<<gw, dim3(256), 0, s>>>(B, c->N, (const float*)eloc_old, (const float*)eloc_new,
                                                  (const float*)grad_eff_old, (const float*)grad_new_eff, tdamp, tstep,
                                                  (const float*)e_trial_b, (const float*)e_est_b, e_trial, e_est,
                                                  cut_minima, cpart, (float*)weights_inout);
  else
    k_dmc_weights<double><<<gw, dim3(256), 0, s>>>(B, c->N, (const double*)eloc_old, (const double*)eloc_new,
                                                   (const double*)grad_eff_old, (const double*)grad_new_eff, tdamp,
                                                   tstep, (const double*)e_trial_b, (const double*)e_est_b, e_trial,
                                                   e_est, cut_minima, cpart, (double*)weights_inout);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_dmc_weights(aiqmc_ctx* c, int32_t B, const void* eloc_old, const void* eloc_new, const void* grad_eff_old,
                      const void* grad_new_eff, const double* tdamp, double tstep, double e_trial, double e_est,
                      double branchcut, void* weights_inout, void* stream) {
  return aiqmc_dmc_weights_ex(c, B, eloc_old, eloc_new, grad_eff_old, grad_new_eff, tdamp, tstep, nullptr, nullptr,
                              e_trial, e_est, branchcut, nullptr, weights_inout, stream);
}

int aiqmc_dmc_cut_minima(aiqmc_ctx* c, int32_t B, const void* eloc_old, const void* eloc_new, const void* e_est_b,
                         double e_est, double branchcut, double* out, void* stream) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (B < 0) return fail(AIQMC_EINVAL, "negative batch");
  if (!out || (B > 0 && (!eloc_old || !eloc_new))) return fail(AIQMC_EINVAL, "null argument");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  double* d = dmc_scratch(c);
  if (!d) return fail(AIQMC_EHIP, "hipMalloc: DMC scratch");
  if (c->dtype == AIQMC_F32)
    k_dmc_cut_part<float><<<dim3(DMC_NB), dim3(256), 0, s>>>(B, (const float*)eloc_old, (const float*)eloc_new,
                                                             (const float*)e_est_b, e_est, branchcut, d);
  else
    k_dmc_cut_part<double><<<dim3(DMC_NB), dim3(256), 0, s>>>(B, (const double*)eloc_old, (const double*)eloc_new,
                                                              (const double*)e_est_b, e_est, branchcut, d);
  k_dmc_cut_fin<<<dim3(1), dim3(64), 0, s>>>(d, out);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_dmc_branch(aiqmc_ctx* c, int32_t B, const void* weights, double u, int32_t* newinds, void* weight_out,
                     void* stream) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (B <= 0) return fail(AIQMC_EINVAL, "empty batch");
  if (!weights || !newinds || !weight_out) return fail(AIQMC_EINVAL, "null argument");
  if (!(u >= 0.0 && u < 1.0)) return fail(AIQMC_EINVAL, "u must be in [0, 1)");
  HIPCHK(hipSetDevice(c->device));
  double* csum = nullptr;
  HIPCHK(hipMallocAsync((void**)&csum, (size_t)B * sizeof(double), (hipStream_t)stream));
  hipStream_t s = (hipStream_t)stream;
  if (c->dtype == AIQMC_F32)
    k_dmc_branch<float><<<dim3(1), dim3(1024), 0, s>>>(B, (const float*)weights, u, csum, newinds, (float*)weight_out);
  else
    k_dmc_branch<double><<<dim3(1), dim3(1024), 0, s>>>(B, (const double*)weights, u, csum, newinds,
                                                         (double*)weight_out);
  HIPCHK(hipFreeAsync(csum, s));
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_energy_stats(const void* e_l, int32_t dtype, int64_t n, double* out, int32_t finalize, void* stream) {
  if (n <= 0) return fail(AIQMC_EINVAL, "empty batch");
  if (!e_l || !out) return fail(AIQMC_EINVAL, "null argument");
  if (dtype != AIQMC_F32 && dtype != AIQMC_F64) return fail(AIQMC_EINVAL, "dtype must be AIQMC_F32 or AIQMC_F64");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == AIQMC_F32)
    k_energy_stats<float><<<dim3(1), dim3(1024), 0, s>>>((const float*)e_l, n, out, finalize != 0);
  else
    k_energy_stats<double><<<dim3(1), dim3(1024), 0, s>>>((const double*)e_l, n, out, finalize != 0);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_loss_weights(const void* e_re, const void* e_im, int32_t dtype, int64_t n, double clip_scale,
                       int32_t center_at_clipped, double wscale, void* w_re, void* w_im, void* clipped_re,
                       void* clipped_im, double* stats, void* stream) {
  if (n <= 0) return fail(AIQMC_EINVAL, "empty batch");
  if (!e_re || !w_re || !stats) return fail(AIQMC_EINVAL, "null argument");
  if (dtype != AIQMC_F32 && dtype != AIQMC_F64) return fail(AIQMC_EINVAL, "dtype must be AIQMC_F32 or AIQMC_F64");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == AIQMC_F32)
    k_loss_weights<float><<<dim3(1), dim3(1024), 0, s>>>((const float*)e_re, (const float*)e_im, n, clip_scale,
                                                         center_at_clipped, wscale, (float*)w_re, (float*)w_im,
                                                         (float*)clipped_re, (float*)clipped_im, stats);
  else
    k_loss_weights<double><<<dim3(1), dim3(1024), 0, s>>>((const double*)e_re, (const double*)e_im, n, clip_scale,
                                                          center_at_clipped, wscale, (double*)w_re, (double*)w_im,
                                                          (double*)clipped_re, (double*)clipped_im, stats);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_energy_stats_final(double* out, void* stream) {
  if (!out) return fail(AIQMC_EINVAL, "null argument");
  k_energy_stats_final<<<dim3(1), dim3(64), 0, (hipStream_t)stream>>>(out);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_profile_enable(aiqmc_ctx* c, int32_t on) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->prof = on != 0;
  return AIQMC_OK;
}

int aiqmc_profile_read(aiqmc_ctx* c, int32_t slot, double* total_ms, int64_t* launches) {
  if (!c || slot < 0 || slot >= AIQMC_PROF_SLOTS || !total_ms || !launches) return fail(AIQMC_EINVAL, "bad argument");
  double tot = 0.0;
  int64_t n = 0;
  for (auto& p : c->ev_used[slot]) {
    HIPCHK(hipEventSynchronize(p.second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    tot += ms;
    ++n;
    c->ev_free.push_back(p.first);
    c->ev_free.push_back(p.second);
  }
  c->ev_used[slot].clear();
  *total_ms = tot;
  *launches = n;
  return AIQMC_OK;
}

int aiqmc_debug_logpsi_grad_forward(aiqmc_ctx* c, const void* pos, int32_t B, void* logabs, void* grad,
                                     void* stream) {
  int rc = check_call(c, pos, B);
  if (rc) return rc;
  if (B == 0) return AIQMC_OK;
  if (!grad) return fail(AIQMC_EINVAL, "null grad");
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  KArgs ka = base_args(c);
  ka.nconf = B;
  ka.pos = pos;
  ka.logabs = logabs;
  ka.grad = grad;
  ops.walker(c->dtype, MODE_GRAD_FWD, ka, B, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return AIQMC_OK;
}

int aiqmc_debug_set_ablate(aiqmc_ctx* c, int32_t mask) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->ablate = mask;
  return AIQMC_OK;
}

int aiqmc_debug_set_lap_waves(aiqmc_ctx* c, int32_t waves) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (waves != 0 && waves != 1 && waves != 2 && waves != 4) return fail(AIQMC_EINVAL, "lap waves must be 0, 1, 2 or 4");
  c->lap_waves = waves;
  return AIQMC_OK;
}

int aiqmc_debug_set_fuse_accept(aiqmc_ctx* c, int32_t on) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->fuse_accept = on != 0;
  return AIQMC_OK;
}

int aiqmc_debug_set_packed_walkers(aiqmc_ctx* c, int32_t on) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->packed_walkers = on != 0;
  return AIQMC_OK;
}

int aiqmc_debug_launch_lds(int32_t nelectrons, int32_t natoms, int32_t dtype, int32_t kind, int32_t* bytes,
                           int32_t* waves) {
  ShapeOps ops{};
  if (!shape_ops(nelectrons, natoms, &ops)) return fail(AIQMC_EUNSUPPORTED, "no kernel instantiation for this shape");
  if (kind < 0 || kind > 5) return fail(AIQMC_EINVAL, "kind must be one of AIQMC_LDS_*");
  if (dtype != AIQMC_F32 && dtype != AIQMC_F64) return fail(AIQMC_EINVAL, "dtype must be AIQMC_F32 or AIQMC_F64");
  const int d = dtype == AIQMC_F32 ? 0 : 1;
  if (bytes) *bytes = ops.dyn_lds[d][kind];
  if (waves) *waves = ops.wg_waves[d][kind];
  return AIQMC_OK;
}

int aiqmc_debug_set_walker_pivots(aiqmc_ctx* c, int32_t reuse) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->walker_fixed_gj = reuse != 0;
  return AIQMC_OK;
}

int aiqmc_debug_set_fuse_reduce(aiqmc_ctx* c, int32_t on) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (on < 0 || on > 3) return fail(AIQMC_EINVAL, "fuse_reduce must be 0, 1, 2 or 3");
  c->fuse_reduce = on == 3 ? 0 : on;
  c->wide_reduce = on == 3 ? 0 : 1;
  return AIQMC_OK;
}

}  // extern "C"

// aiqmc_debug_limdrift_factor: the fused path's per-configuration accumulation (tacc_add, one
// thread per configuration instead of lane 0 of its wave) and the consumers' read (taueff_wave).
__global__ __launch_bounds__(256) void k_tacc_feed(const float* __restrict__ x, int n, unsigned long long* acc) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i < n) tacc_add(acc, 0, i, (double)x[i]);
}
__global__ __launch_bounds__(64) void k_taueff_read(const unsigned long long* acc, const unsigned long long* part,
                                                    double tstep, double* out) {
  const float te = taueff_wave<float>(nullptr, acc, 0, tstep, part);
  if (threadIdx.x == 0) *out = (double)te;
}

extern "C" {

int aiqmc_debug_limdrift_factor(aiqmc_ctx* c, const void* sumsq, int32_t n, double tstep, int32_t mode, double* out,
                                void* stream) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  if (!sumsq || !out || n <= 0) return fail(AIQMC_EINVAL, "limdrift_factor: null buffer or n <= 0");
  if (n >= TACC_MAX_CONF && mode != 2) return fail(AIQMC_EINVAL, "limdrift_factor: n >= 2^24 needs mode 2");
  if (mode < 0 || mode > 2) return fail(AIQMC_EINVAL, "limdrift_factor: mode must be 0, 1 or 2");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const size_t words = (size_t)TACC_STRIDE + TPART_KIND + 1;   // acc | part | out (as a double)
  unsigned long long* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, words * sizeof(unsigned long long)));
  unsigned long long* acc = d;
  unsigned long long* part = d + TACC_STRIDE;
  double* dout = (double*)(d + TACC_STRIDE + TPART_KIND);
  int rc = AIQMC_OK;
  if (hipMemsetAsync(d, 0, words * sizeof(unsigned long long), s) != hipSuccess) rc = fail(AIQMC_EHIP, "memset");
  if (!rc) {
    const float* x = (const float*)sumsq;
    if (mode == 0) {
      k_tacc_feed<<<dim3((n + 255) / 256), dim3(256), 0, s>>>(x, n, acc);
      k_taueff_read<<<dim3(1), dim3(64), 0, s>>>(acc, nullptr, tstep, dout);
    } else if (mode == 1) {
      k_taueff_part<<<dim3(TPART), dim3(256), 0, s>>>(x, n, part);
      k_taueff_read<<<dim3(1), dim3(64), 0, s>>>(nullptr, part, tstep, dout);
    } else {
      k_taueff<float><<<dim3(1), dim3(1024), 0, s>>>(x, n, tstep, dout);
    }
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(out, dout, sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = fail(AIQMC_EHIP, "limdrift_factor: launch or copy");
  }
  (void)hipFree(d);
  return rc;
}

int aiqmc_debug_set_proposal_reuse(aiqmc_ctx* c, int32_t on) {
  if (!c) return fail(AIQMC_EINVAL, "null context");
  c->reuse = on != 0;
  return AIQMC_OK;
}

int aiqmc_debug_phase_cycles(aiqmc_ctx* c, uint64_t* out32) {
  if (!c || !out32) return fail(AIQMC_EINVAL, "null argument");
  ShapeOps ops;
  shape_ops(c->N, c->A, &ops);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());
  ops.phase_read((unsigned long long*)out32);
  return AIQMC_OK;
}

}  // extern "C"
