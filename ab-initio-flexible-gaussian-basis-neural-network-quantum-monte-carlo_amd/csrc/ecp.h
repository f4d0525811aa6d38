// ecp.h -- pseudopotential (ccECP) local energy of the AIQMC wavefunction
// (AIQMCrelease3/Energy/pphamiltonian.py:130-190, pseudopotential/pseudopotential.py:86-318,
// pseudopotential/pp_energy_test.py:45-105).
//
// Per walker b the nonlocal part needs log psi at N*A*50 configurations: electron i moved to
// r_ia * (p_q R_b), p_q the 50-point octahedral grid (pseudopotential.py:181-225), R_b the
// walker's random orthogonal matrix (get_rot :233-241).  Each of them differs from the walker
// in ONE electron, so they run through the Metropolis proposal machinery (walker_rev.h): the
// walker launch writes the walker cache, k_moved_electron the moved electron's stage, and a
// value-only proposal launch of k_walker_rev patches the pair sums and reuses the walker's
// Gauss-Jordan pivot order.  Kernels here:
//   k_ecp_rot     Haar O(3) matrix per walker from Philox (production draws)
//   k_ecp_points  moved-electron positions x' = r_ia p_q R_b, one thread per configuration
//   k_ecp_energy  one wave per walker: local pp part, sum_{i,a,q} P_l(cos) v_l(r) ratio,
//                 added to the all-electron local energy of the same walker
// Reference quirks (oracle/pphamiltonian.py E1-E7) are reproduced; the ECP arithmetic itself is
// done in double for both dtypes (it is < 1% of the launch time).
#pragma once
#include "jets.h"

namespace aq {

constexpr int ECP_NQ = 50;   // 6 (OA) + 12 (OB) + 8 (OC) + 24 (OD) points

// Grid points in the reference's order and its 8-digit literals (pseudopotential.py:197-223).
__device__ __forceinline__ void ecp_point(int q, double p[3], int& grp) {
  const double s2 = 0.70710678, s3 = 0.57735027;
  if (q < 6) {
    grp = 0;
    const int ax[6] = {0, 1, 2, 2, 1, 0};
    const double sg[6] = {-1.0, -1.0, -1.0, 1.0, 1.0, 1.0};
    p[0] = p[1] = p[2] = 0.0;
    p[ax[q]] = sg[q];
    return;
  }
  if (q < 18) {
    grp = 1;
    // OB rows: (-,-,0) (-,0,-) (-,0,+) (-,+,0) (0,-,-) (0,-,+) (0,+,-) (0,+,+) (+,-,0) (+,0,-) (+,0,+) (+,+,0)
    const signed char t[12][3] = {{-1, -1, 0}, {-1, 0, -1}, {-1, 0, 1}, {-1, 1, 0}, {0, -1, -1}, {0, -1, 1},
                                  {0, 1, -1},  {0, 1, 1},   {1, -1, 0}, {1, 0, -1}, {1, 0, 1},  {1, 1, 0}};
    for (int d = 0; d < 3; ++d) p[d] = t[q - 6][d] * s2;
    return;
  }
  // OC rows in binary order of (x, y, z) signs, - before +
  const int c = q < 26 ? q - 18 : (q - 26) % 8;
  double o[3] = {(c & 4) ? s3 : -s3, (c & 2) ? s3 : -s3, (c & 1) ? s3 : -s3};
  if (q < 26) {
    grp = 2;
    for (int d = 0; d < 3; ++d) p[d] = o[d];
    return;
  }
  // OD = [OD1; OD2; OD3], d1 = OC sqrt(3/11), component 2 / 1 / 0 tripled (:219-223)
  grp = 3;
  const double f = sqrt(3.0 / 11.0);
  const int tri = 2 - (q - 26) / 8;
  for (int d = 0; d < 3; ++d) p[d] = (o[d] * f) * (d == tri ? 3.0 : 1.0);
}

__device__ __forceinline__ int ecp_group_begin(int g) { return g == 0 ? 0 : (g == 1 ? 6 : (g == 2 ? 18 : 26)); }
__device__ __forceinline__ int ecp_group_end(int g) { return g == 0 ? 6 : (g == 1 ? 18 : (g == 2 ? 26 : 50)); }
__device__ __forceinline__ double ecp_weight(int g) {
  return g == 0 ? 4.0 / 315.0 : (g == 1 ? 64.0 / 2835.0 : (g == 2 ? 27.0 / 1280.0 : 14641.0 / 725760.0));
}

// p' = p R  (einsum 'jkl,ik->jil', pseudopotential.py:237-240), R row-major [k][l]
template <typename T>
__device__ __forceinline__ void ecp_rotate(const T* R, const double p[3], double out[3]) {
#pragma unroll
  for (int l = 0; l < 3; ++l) out[l] = p[0] * (double)R[l] + p[1] * (double)R[3 + l] + p[2] * (double)R[6 + l];
}

// Device tables (double): atoms [A][3], charges [A], then per atom KL local triplets
// (n, coefficient, exponent) and L*KN nonlocal triplets.
struct EcpArgs {
  int B, N, A, KL, KN, L;
  const double* tab;
  const void* pos;      // [B][3N]
  const void* rot;      // [B][9]
  const void* lp0;      // [B] log|psi| at the walker
  const void* ph0;      // [B] phase at the walker
  const void* lpq;      // [B][N][A][50] log|psi| at the quadrature configurations
  const void* phq;      // [B][N][A][50] phase
  const void* eall;     // [B] all-electron local energy (V_ee + V_en + V_nn + KE)
  void* e_re;           // [B] outputs
  void* e_im;
  void* xnew;           // k_ecp_points output [B*N*A*50][3]
  uint64_t seed, step;  // k_ecp_rot
  int skip_nl;          // k_ecp_energy: nonlocal coefficients all zero -- no quadrature was run
  int cdf_lds;          // k_tmove: dynamic LDS holds every electron's cdf row [N][A*50+1][2]
  // T-moves (k_tmove)
  double tstep;
  const void* usel;     // [B] selection uniform (NULL: Philox)
  const void* uacc;     // [B][N] acceptance uniforms (NULL: Philox)
  void* acc;            // [B][N] acceptance out (optional)
  void* pos_out;        // [B][3N] positions, updated in place
  double* scr;          // [B][N*A*50][4] forward amplitude (re, im), ratio (re, im)
};

// Uniform Haar O(3): a uniformly random unit quaternion (4 normals, normalised) gives SO(3);
// an independent fair sign makes it O(3), the support of jax.random.orthogonal.
template <typename T>
__global__ __launch_bounds__(256) void k_ecp_rot(EcpArgs ea) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= ea.B) return;
  float g[3], h[3], u[4];
  philox_normal3f(ea.seed, ea.step, (uint32_t)b, 16u, g);
  philox_normal3f(ea.seed, ea.step, (uint32_t)b, 17u, h);
  philox_u4(ea.seed, ea.step, (uint32_t)b, 18u, u);
  double w = g[0], x = g[1], y = g[2], z = h[0];
  const double n = 1.0 / sqrt(w * w + x * x + y * y + z * z);
  w *= n; x *= n; y *= n; z *= n;
  const double s = u[0] < 0.5f ? -1.0 : 1.0;
  const double m[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w),     2 * (x * z + y * w),
                       2 * (x * y + z * w),     1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                       2 * (x * z - y * w),     2 * (y * z + x * w),     1 - 2 * (x * x + y * y)};
  T* R = (T*)ea.rot + (size_t)b * 9;
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = (T)(s * m[k]);
}

// x'[conf] = r_ia p_q R_b with conf = ((b N + i) A + a) 50 + q  (E2: not offset by R_a)
template <typename T>
__global__ __launch_bounds__(256) void k_ecp_points(EcpArgs ea) {
  const int M = ea.N * ea.A * ECP_NQ;
  const size_t conf = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (conf >= (size_t)ea.B * M) return;
  const int b = (int)(conf / M);
  const int rem = (int)(conf - (size_t)b * M);
  const int i = rem / (ea.A * ECP_NQ);
  const int a = (rem / ECP_NQ) % ea.A;
  const int q = rem % ECP_NQ;
  const T* x = (const T*)ea.pos + (size_t)b * 3 * ea.N + 3 * i;
  double r2 = 0.0;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const double t = (double)x[d] - ea.tab[a * 3 + d];
    r2 += t * t;
  }
  const double r = sqrt(r2);
  double p[3], pr[3];
  int grp;
  ecp_point(q, p, grp);
  ecp_rotate<T>((const T*)ea.rot + (size_t)b * 9, p, pr);
  T* o = (T*)ea.xnew + conf * 3;
#pragma unroll
  for (int d = 0; d < 3; ++d) o[d] = (T)(r * pr[d]);
}

__device__ __forceinline__ double ecp_radial(const double* t, int K, double r, double nshift) {
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += t[3 * k + 1] * pow(r, t[3 * k] + nshift) * exp(-t[3 * k + 2] * r * r);
  return s;
}

// P_l(x) of pseudopotential.py:250-269 (1/(4 pi) included, E5)
__device__ __forceinline__ double ecp_pl(int l, double x) {
  const double c = 0.079577471545947668;   // 1/(4 pi)
  if (l == 0) return c;
  if (l == 1) return 3.0 * c * x;
  if (l == 2) return 5.0 * c * 0.5 * (3.0 * x * x - 1.0);
  return 7.0 * c * 0.5 * (5.0 * x * x * x - 3.0 * x);
}

// E3's Frobenius norm of a grid group's rotated coordinates r p'_q is r^2 F_g with
// F_g = sum_{q in g} |p_q R|^2, which depends on the walker's rotation only: one point per lane,
// four masked wave sums (instead of a loop over the group's points for every quadrature entry).
template <typename T>
__device__ __forceinline__ void ecp_group_norms(const T* R, int lane, double Fg[4]) {
  double v = 0.0;
  int gl = -1;
  if (lane < ECP_NQ) {
    double p[3], pr[3];
    ecp_point(lane, p, gl);
    ecp_rotate<T>(R, p, pr);
    v = pr[0] * pr[0] + pr[1] * pr[1] + pr[2] * pr[2];
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) Fg[g] = wave_sum(gl == g ? v : 0.0);
}

// The nonlocal radial factors v_l(r_ia) (pseudopotential.py:118-160) of every (electron, atom)
// pair, once per pair instead of once per quadrature point (they do not depend on the point: fp64
// pow and exp per term were ≈ 90 % of the launch's instructions); the same arithmetic, so the same
// bits.  tm = 0: v_l; tm != 0: exp(-tstep v_l) - 1 (the T-move amplitude factor, T2).
constexpr int ECP_MAXPAIR = 64;   // N A of every built shape (16 x 3, 10 x 5)
template <typename T>
__device__ __forceinline__ void ecp_pair_radials(const EcpArgs& ea, const T* x, int lane, double (*vl)[4], bool tm) {
  const int N = ea.N, A = ea.A;
  const int stride = 3 * (ea.KL + ea.L * ea.KN);
  const double* atoms = ea.tab;
  const double* tabs = ea.tab + 4 * A;
  for (int j = lane; j < N * A; j += 64) {
    const int i = j / A, a = j - (j / A) * A;
    double r2 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const double t = (double)x[3 * i + d] - atoms[a * 3 + d];
      r2 += t * t;
    }
    const double r = sqrt(r2);
    const double* tnl = tabs + a * stride + 3 * ea.KL;
    for (int l = 0; l < ea.L; ++l) {
      const double v = ecp_radial(tnl + 3 * ea.KN * l, ea.KN, r, 0.0);
      vl[j][l] = tm ? exp(-ea.tstep * v) - 1.0 : v;
    }
  }
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(64) void k_ecp_energy(EcpArgs ea) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = ea.N, A = ea.A;
  const int M = N * A * ECP_NQ;
  const double* atoms = ea.tab;
  const double* charges = ea.tab + 3 * A;
  const int stride = 3 * (ea.KL + ea.L * ea.KN);
  const double* tabs = ea.tab + 4 * A;
  const T* x = (const T*)ea.pos + (size_t)b * 3 * N;
  const T* R = (const T*)ea.rot + (size_t)b * 9;
  double Fg[4] = {0.0, 0.0, 0.0, 0.0};
  if (!ea.skip_nl) ecp_group_norms<T>(R, lane, Fg);   // skip_nl: no rotations drawn
  const double la0 = ea.skip_nl ? 1.0 : (double)((const T*)ea.lp0)[b];
  const double ph0 = ea.skip_nl ? 0.0 : (double)((const T*)ea.ph0)[b];
  const double dn = 1.0 / (la0 * la0 + ph0 * ph0);   // 1 / den, den = la0 + i ph0 (E4)
  double er = 0.0, ei = 0.0;
  __shared__ double vl[ECP_MAXPAIR][4];
  const bool pair_tab = N * A <= ECP_MAXPAIR && ea.L <= 4;
  if (pair_tab && !ea.skip_nl) ecp_pair_radials<T>(ea, x, lane, vl, false);
  // zero nonlocal coefficients: every term is v_l(r) = 0 times a finite ratio, exactly 0
  for (int idx = ea.skip_nl ? M : lane; idx < M; idx += 64) {
    const int i = idx / (A * ECP_NQ);
    const int a = (idx / ECP_NQ) % A;
    const int q = idx % ECP_NQ;
    double ae[3], r2 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      ae[d] = (double)x[3 * i + d] - atoms[a * 3 + d];
      r2 += ae[d] * ae[d];
    }
    const double r = sqrt(r2);
    double p[3], pr[3];
    int grp;
    ecp_point(q, p, grp);
    ecp_rotate<T>(R, p, pr);
    // Frobenius norm of the group's rotated coordinates r p'_q (E3)
    const double fro2 = r * r * Fg[grp];
    const double dot = ae[0] * (r * pr[0]) + ae[1] * (r * pr[1]) + ae[2] * (r * pr[2]);
    const double cs = dot / (r * sqrt(fro2));
    const size_t conf = (size_t)b * M + idx;
    const double la = (double)((const T*)ea.lpq)[conf], ph = (double)((const T*)ea.phq)[conf];
    const double w = ecp_weight(grp);
    // ratio = (la + i ph) / (la0 + i ph0) * w
    const double rr = (la * la0 + ph * ph0) * dn * w, ri = (ph * la0 - la * ph0) * dn * w;
    const double* tnl = tabs + a * stride + 3 * ea.KL;
    double s = 0.0;
    for (int l = 0; l < ea.L; ++l)
      s += ecp_pl(l, cs) * (pair_tab ? vl[i * A + a][l] : ecp_radial(tnl + 3 * ea.KN * l, ea.KN, r, 0.0));   // E1
    er += s * rr;
    ei += s * ri;
  }
  // local part: -Z_a / r_ia + sum_k c r^(n-2) e^{-alpha r^2}  (pseudopotential.py:95-116)
  for (int idx = lane; idx < N * A; idx += 64) {
    const int i = idx / A, a = idx - (idx / A) * A;
    double r2 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const double t = (double)x[3 * i + d] - atoms[a * 3 + d];
      r2 += t * t;
    }
    const double r = sqrt(r2);
    er += -charges[a] / r + ecp_radial(tabs + a * stride, ea.KL, r, -2.0);
  }
  er = wave_sum(er);
  ei = wave_sum(ei);
  if (lane == 0) {
    // the all-electron E_L carries -sum Z/r already; the pp Hamiltonian has it once, in the
    // local part (E7): remove the all-electron copy
    double ven = 0.0;
    for (int i = 0; i < N; ++i)
      for (int a = 0; a < A; ++a) {
        double r2 = 0.0;
        for (int d = 0; d < 3; ++d) {
          const double t = (double)x[3 * i + d] - atoms[a * 3 + d];
          r2 += t * t;
        }
        ven -= charges[a] / sqrt(r2);
      }
    ((T*)ea.e_re)[b] = (T)((double)((const T*)ea.eall)[b] - ven + er);
    ((T*)ea.e_im)[b] = (T)ei;
  }
}

// Acceptance of T-moves with zero nonlocal coefficients: every amplitude is 0, norm = back norm
// = 1, nothing moves and the acceptance is exactly 1 (what k_tmove computes for such tables).
template <typename T>
__global__ __launch_bounds__(256) void k_tmove_none(T* __restrict__ acc, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) acc[t] = T(1);
}

// T-moves (DMC/Tmoves.py:68-224; oracle/dmc.py tmoves, quirks T1-T8), one wave per walker.
// Pass 1 (lanes over the N*A*50 quadrature entries): ratio (E4, times w_g), t_amp = ratio *
// sum_l (exp(-tau v_l) - 1) P_l(cos), forward amplitude = lexicographic max(t_amp, 0), and the
// walker's norm 1 + sum w_g fwd.  Pass 2 (lanes over electrons): the scan binary search of
// jnp.searchsorted on the row cdf (prefix sums recomputed per probe: rows are <= A*50+1 long),
// back norm over the hard-coded slices, acceptance, in-place move from the original position.
__device__ __forceinline__ bool cplx_le(double qr, double qi, double ar, double ai) {
  return qr < ar || (qr == ar && qi <= ai);
}

template <typename T>
__global__ __launch_bounds__(64) void k_tmove(EcpArgs ea) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = ea.N, A = ea.A;
  const int AQ = A * ECP_NQ, M = N * AQ, M1 = AQ + 1;
  const double* atoms = ea.tab;
  const int stride = 3 * (ea.KL + ea.L * ea.KN);
  const double* tabs = ea.tab + 4 * A;
  const T* x = (const T*)ea.pos + (size_t)b * 3 * N;
  const T* R = (const T*)ea.rot + (size_t)b * 9;
  double Fg[4];
  ecp_group_norms<T>(R, lane, Fg);
  const double la0 = (double)((const T*)ea.lp0)[b], ph0 = (double)((const T*)ea.ph0)[b];
  const double dn = 1.0 / (la0 * la0 + ph0 * ph0);
  double* scr = ea.scr + (size_t)b * M * 4;
  double nr = 0.0, ni = 0.0;
  __shared__ double el[ECP_MAXPAIR][4];
  const bool pair_tab = N * A <= ECP_MAXPAIR && ea.L <= 4;
  if (pair_tab) ecp_pair_radials<T>(ea, x, lane, el, true);
  for (int idx = lane; idx < M; idx += 64) {
    const int i = idx / AQ;
    const int a = (idx / ECP_NQ) % A;
    const int q = idx % ECP_NQ;
    double ae[3], r2 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      ae[d] = (double)x[3 * i + d] - atoms[a * 3 + d];
      r2 += ae[d] * ae[d];
    }
    const double r = sqrt(r2);
    double p[3], pr[3];
    int grp;
    ecp_point(q, p, grp);
    ecp_rotate<T>(R, p, pr);
    const double fro2 = r * r * Fg[grp];   // E3
    const double dot = ae[0] * (r * pr[0]) + ae[1] * (r * pr[1]) + ae[2] * (r * pr[2]);
    const double cs = dot / (r * sqrt(fro2));
    const size_t conf = (size_t)b * M + idx;
    const double la = (double)((const T*)ea.lpq)[conf], ph = (double)((const T*)ea.phq)[conf];
    const double w = ecp_weight(grp);
    const double rr = (la * la0 + ph * ph0) * dn * w, ri = (ph * la0 - la * ph0) * dn * w;   // T1
    const double* tnl = tabs + a * stride + 3 * ea.KL;
    double wt = 0.0;
    for (int l = 0; l < ea.L; ++l)
      wt += (pair_tab ? el[i * A + a][l] : exp(-ea.tstep * ecp_radial(tnl + 3 * ea.KN * l, ea.KN, r, 0.0)) - 1.0) *
            ecp_pl(l, cs);   // T2
    const double tr = rr * wt, ti = ri * wt;
    const bool pos = tr > 0.0 || (tr == 0.0 && ti > 0.0);   // T3
    const double fr = pos ? tr : 0.0, fi = pos ? ti : 0.0;
    scr[4 * idx + 0] = fr;
    scr[4 * idx + 1] = fi;
    scr[4 * idx + 2] = rr;
    scr[4 * idx + 3] = ri;
    nr += w * fr;   // T4
    ni += w * fi;
  }
  nr = 1.0 + wave_sum(nr);
  ni = wave_sum(ni);
  __threadfence_block();
  __syncthreads();
  double us;
  if (ea.usel) {
    us = (double)((const T*)ea.usel)[b];
  } else {
    float u[4];
    philox_u4(ea.seed, ea.step, (uint32_t)b, 19u, u);
    us = (double)u[0] - 5.9604644775390625e-08;   // (0,1] -> [0,1)
  }
  const double qr = us + 1.0;
  const double in2 = 1.0 / (nr * nr + ni * ni);
  const double inr = nr * in2, ini = -ni * in2;   // 1 / norm
  int levels = 0;
  while ((1 << levels) < M1 + 1) ++levels;        // ceil(log2(M1 + 1))
  const int lo_[5] = {0, 1, 19, 55, 79}, hi_[5] = {1, 19, 55, 79, 151};
  extern __shared__ double cdf_s[];   // cdf_lds: [N][M1][2]
  for (int e = lane; e < N; e += 64) {
    // T5: jnp.searchsorted(cdf_e, u + 1), cdf_e[k] = sum_{j<=k} row_e[j] / norm
    const double* fe = scr + (size_t)e * AQ * 4;
    int low = 0, high = M1;
    if (ea.cdf_lds) {
      // the row's cdf once, in the same order of operations as the per-probe sums below (so the
      // same bits), then the search reads it: one pass over the row instead of one per probe
      double* ce = cdf_s + (size_t)e * M1 * 2;
      double cr = inr, ci = ini;
      ce[0] = cr;
      ce[1] = ci;
      for (int j = 1; j < M1; ++j) {
        const double fr = fe[4 * (j - 1)], fi = fe[4 * (j - 1) + 1];
        cr += fr * inr - fi * ini;
        ci += fr * ini + fi * inr;
        ce[2 * j] = cr;
        ce[2 * j + 1] = ci;
      }
      for (int lv = 0; lv < levels; ++lv) {
        const int mid = (low + high) >> 1;
        if (cplx_le(qr, 0.0, ce[2 * mid], ce[2 * mid + 1])) high = mid;
        else low = mid;
      }
    } else
    for (int lv = 0; lv < levels; ++lv) {
      const int mid = (low + high) >> 1;
      double cr = inr, ci = ini;   // row_e[0] = 1
      for (int j = 1; j <= mid; ++j) {
        const double fr = fe[4 * (j - 1)], fi = fe[4 * (j - 1) + 1];
        cr += fr * inr - fi * ini;
        ci += fr * ini + fi * inr;
      }
      if (cplx_le(qr, 0.0, cr, ci)) high = mid;
      else low = mid;
    }
    const int mv = high < M1 ? high : 0;
    // T6: back amplitudes = row[min(mv, N-1)] / ratio_total[e, mv]
    double cr = 1.0, ci = 0.0;
    if (mv > 0) {
      const double rr = fe[4 * (mv - 1) + 2], ri = fe[4 * (mv - 1) + 3];
      const double d = 1.0 / (rr * rr + ri * ri);
      cr = rr * d;
      ci = -ri * d;
    }
    const int ri_ = mv < N - 1 ? mv : N - 1;
    const double* fb = scr + (size_t)ri_ * AQ * 4;
    double sr = 0.0, si = 0.0;   // T7: sum_k W_k sum row[slice_k], W_0 = 0
    for (int k = 1; k < 5; ++k) {
      const double wk = ecp_weight(k - 1);
      const int hi = hi_[k] < M1 ? hi_[k] : M1;
      double tr = 0.0, ti = 0.0;
      for (int j = lo_[k]; j < hi; ++j) {
        tr += fb[4 * (j - 1)];
        ti += fb[4 * (j - 1) + 1];
      }
      sr += wk * tr;
      si += wk * ti;
    }
    const double br = 1.0 + (sr * cr - si * ci), bi = sr * ci + si * cr;
    const double acc = (nr * br + ni * bi) / (br * br + bi * bi);   // T8: Re(norm / back_norm)
    double ua;
    if (ea.uacc) {
      ua = (double)((const T*)ea.uacc)[(size_t)b * N + e];
    } else {
      float u[4];
      philox_u4(ea.seed, ea.step, (uint32_t)(b * N + e), 20u, u);
      ua = (double)u[0] - 5.9604644775390625e-08;
    }
    if (ea.acc) ((T*)ea.acc)[(size_t)b * N + e] = (T)acc;
    if (acc > ua && mv > 0) {
      const int m = mv - 1, a = m / ECP_NQ, q = m % ECP_NQ;
      double r2 = 0.0;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const double t = (double)x[3 * e + d] - atoms[a * 3 + d];
        r2 += t * t;
      }
      const double r = sqrt(r2);
      double p[3], pr[3];
      int grp;
      ecp_point(q, p, grp);
      ecp_rotate<T>(R, p, pr);
      T* xo = (T*)ea.pos_out + (size_t)b * 3 * N + 3 * e;
#pragma unroll
      for (int d = 0; d < 3; ++d) xo[d] = (T)(r * pr[d]);   // E2
    }
  }
}

}  // namespace aq
