// walker_rev.h -- reverse-mode value + gradient of log|psi| for ONE configuration
// per wavefront (the Metropolis hot path: VMCmcstep.py:41-53 and :79 evaluate
// jax.grad(logabs) at the walkers and at all B*N single-electron proposals).
//
// Forward pass (values) with lanes over work items, intermediates in LDS:
//   F1 per-electron stage as forward jets along the lane's own coordinate
//      (direction lanes keep d(features)/dx_e and d(Yt row)/dx_e in registers:
//      these sub-Jacobians are local to electron e);
//   F2 pair stream h2[k,i] for all N^2 pairs (lanes over pairs), J_ee, V_ee;
//   F3 spin-group column means g2 (nn.py:151); F4 three h-stream layers
//      (lanes over (electron, unit)); F5 Phi, A = Phi * Yt, Gauss-Jordan -> B.
// Backward pass:
//   B1 dL/dH[r,f] = Re Q_f[r,r] = Re sum_c W_{s(r)}[f,c] Yt[r,c] B[c,r],
//      dL/dYt[r,c] = Re(B[c,r] Phi[r,c]);
//   B2 back through the three h-stream layers (tanh, conv quads, group means);
//   B3 back through each pair's two double layers to d = x_i - x_k (+ J_ee);
//   B4 direction lane (c,e) assembles dlogpsi/dx_{e,c} from pair adjoints and
//      its electron-local sub-Jacobians (Yt row, ae features, J_ae).
#pragma once
#include "jets.h"
#include "layout.h"
#include "walker_kernel.h"
#include "gj.h"
#include "electron.h"

namespace aq {

// Diagnostics build (-DAQ_PHASE_PROF): per-phase shader-clock cycles summed over
// waves, [0..15] walker launches, [16..31] proposal launches (aiqmc_debug_phase_cycles).
#ifdef AQ_PHASE_PROF
static __device__ unsigned long long aq_phase_cycles[32];
#define AQ_PH(k)                                                                         \
  do {                                                                                   \
    const unsigned long long t_ = __builtin_readcyclecounter();                          \
    if (lane == 0) atomicAdd(&aq_phase_cycles[(ka.proposal ? 16 : 0) + (k)], t_ - t_ph); \
    t_ph = t_;                                                                           \
  } while (0)
#elif defined(AQ_PHASE_MARK)
// ISA-inspection build: a marker comment in the assembly at each phase boundary
#define AQ_PH(k) asm volatile(";AQMARK " #k)
#elif defined(AQ_STOP_AFTER)
// register-pressure probe (never a product build): the proposal path ends after phase k, its
// live LDS state kept alive by one store, so the compiled VGPR count is the peak up to phase k
#define AQ_PH(k)                                                                     \
  do {                                                                               \
    if constexpr (PROP && (k) == AQ_STOP_AFTER) {                                    \
      if (ka.logabs) ((T*)ka.logabs)[conf * 64 + lane] = sm[lane] + sm[lane + 1024]; \
      return;                                                                        \
    }                                                                                \
  } while (0)
#else
#define AQ_PH(k) \
  do {           \
  } while (0)
#endif

// Development builds (-DAQ_ABLATE): KArgs.ablate skips phases of the proposal path, so that the
// marginal cost of each phase can be timed (results are garbage; never in a product build).
#ifdef AQ_ABLATE
#define AQ_ABL(b) (isprop && (ka.ablate & (b)))
#else
#define AQ_ABL(b) false
#endif

// FWDREG (proposal instantiations with AQ_FWD_REG): the conv and single-layer outputs of F4 stay
// in registers until B2 instead of the cq / sv blocks (1.68 KB less LDS per wave for N2).
// Round 4, interleaved A/B on one box (N2, 4096 walkers, µs per proposal launch): 219.2-221.7
// with the LDS blocks, 217.9-218.8 with registers (96 VGPRs, no spill; the same 5 waves/SIMD).
// The LDS saving would allow 6 waves/SIMD, but at the 80-VGPR budget that needs, the kernel spills
// 19 VGPRs and measured 230.0-231.1 (profiles/r04_s3_ab_fwdreg.txt).
#ifndef AQ_NO_FWD_REG
constexpr bool kFwdReg = true;
#else
constexpr bool kFwdReg = false;
#endif
template <typename T, int N, int A, bool FWDREG = false, bool COMPACT = false>
struct SmemRev {
  static constexpr int D0 = 4 * A;               // layer-0 h width
  static constexpr int DFM = 3 * D0 + 8;         // widest conv input (layer 0)
  static constexpr int QM = DFM / 4;
  static constexpr int hl_n = N * D0 + N * 4;     // h^0 and h^3 (h^1, h^2 stay in registers)
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  static constexpr int xs = 0;                   // 48
  static constexpr int hl = 48;                  // h^0 [N][D0], h^3 [N][4] (F1..F5)
  static constexpr int hbar = hl;                // their adjoints, same layout (B1..B4)
  static constexpr int QL = (3 * 4 + 8) / 4;     // conv outputs of layers 1, 2
  static constexpr int cq = hl + hl_n;           // conv outputs (kept for backward): [N][QM], [2][N][QL]
  static constexpr int sv = cq + (FWDREG ? 0 : N * QM + 2 * N * QL);   // [3][N][4]   single outputs
  static constexpr int cqo(int l, int i) { return l == 0 ? i * QM : N * QM + ((l - 1) * N + i) * QL; }
  static constexpr int g2 = sv + (FWDREG ? 0 : 3 * N * 4);   // [3][2][N][4] g2 values (forward) / adjoints (backward)
  static constexpr int yv = g2 + 3 * 2 * N * 4;  // [N][N]  Yt (F1..B1)
  static constexpr int ybar = yv;                // [N][N]  its adjoint (B1..B4)
  // region R, lifetimes disjoint: reuse scratch (F0..F2) -> {Phi [N][N][2], B [N][N][2]} (F5..B1)
  // -> dbar [N][N][3] (B3..B4)
  static constexpr int R = yv + N * N;
  // COMPACT (the 7-waves/SIMD proposal instantiation): Phi stays in registers (F5 -> B1), B alone
  // in R, and F2's pair-patch scratch holds new - old differences [32][12] instead of the four parts
  // [64][12]: 5.6 KB per wave for N2 (28 waves/CU fit the 160 KB)
  static constexpr int ph = R;
  static constexpr int mx = COMPACT ? R : R + N * N * 2;
  static constexpr int dbar = R;
  static constexpr int R_n = COMPACT ? cmax(cmax(2 * N * N, 3 * N * N), 4 + 32 * 12)
                                     : cmax(cmax(4 * N * N, 3 * N * N), 4 + 64 * 12);
  // the walker's pivot record [2N+2] (proposals; [3N+2] walker launches) lives in the g2 region during F5: the g2
  // values are dead after F4 and their adjoints are written from B2 on
  static constexpr int pv = g2;
  // proposals: F5's slot table after the pivot record, [4 RW slots][4] ints (Yt row offset, the
  // h^3 row offset for each half of the spin-stacked orbital weights, flag), then a zero row
  static constexpr int RW = (N + 3) / 4;
  static constexpr int st = ((g2 + 3 * N + 2 + 3) / 4) * 4;
  static constexpr int zr = st + (4 * RW * 4 * 4 + (int)sizeof(T) - 1) / (int)sizeof(T);
  static_assert(zr + 4 <= g2 + 3 * 2 * N * 4, "slot table outside the g2 region");
  // FWDREG (proposals): the e-n Jastrow gradient of the direction lanes, parked from F2 to B4
  static constexpr int jdo = R + R_n;
  static constexpr int end = jdo + (FWDREG ? 64 : 0);
  static constexpr int bytes = ((end * (int)sizeof(T)) + 15) & ~15;
  static constexpr int hoff(int l) { return l == 0 ? 0 : N * D0; }   // l = 0 or 3
};

// Per-walker cache written by the walker launch of a Metropolis sweep and read by
// the N single-electron proposals of that walker (they differ from it in one
// electron): electron-local stage of every electron and the spin-group column
// sums of the pair stream.
template <int N, int A>
struct WCache {
  static constexpr int D0 = 4 * A;
  static constexpr int yv = 0;                      // [N][N]     Yt values
  static constexpr int h0 = yv + N * N;             // [N][D0]    ae features
  static constexpr int loc = h0 + N * D0;           // [N+D0][48] electron-local Jacobians
  static constexpr int jaev = loc + (N + D0) * 48;  // [N]        J_ae per electron
  static constexpr int jaed = jaev + N;             // [48]       dJ_ae/dx per direction lane
  static constexpr int g2 = jaed + 48;              // [3][2][N][4]
  static constexpr int jee = g2 + 3 * 2 * N * 4;    // [1]        J_ee
  static constexpr int pv = jee + 1;                // [3N+2]     Gauss-Jordan pivot record (gj.h)
  static constexpr int pt = ((pv + 3 * N + 2 + 3) / 4) * 4; // [N][N][8]  tanh outputs t1, t2 of pair (k, i)
  static constexpr int size = ((pt + 8 * N * N + 63) / 64) * 64;
};
// Per-proposal electron-local stage of the moved electron (k_moved_electron).
template <int N, int A>
struct ECache {
  static constexpr int D0 = 4 * A;
  static constexpr int yv = 0;          // [N]     Yt row values
  static constexpr int h0 = N;          // [D0]    ae features
  static constexpr int yd = N + D0;     // [3][N]  dYt/dx_c
  static constexpr int hd = yd + 3 * N; // [3][D0] dfeat/dx_c
  static constexpr int jv = hd + 3 * D0;
  static constexpr int jd = jv + 1;     // [3]
  static constexpr int xp = jd + 3;     // [3]     the moved electron's proposed position
  static constexpr int size = ((xp + 3 + 15) / 16) * 16;
};

template <typename T, int N, int A>
__device__ __forceinline__ void pair_values(const T d[3], cptr<T> P, T out[3][4]) {
  using Ly = Lay<N, A>;
  const T RSQ2 = T(0.70710678118654752);
  T p[4];
  p[0] = f_sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
#pragma unroll
  for (int c = 0; c < 3; ++c) p[1 + c] = d[c];
#pragma unroll
  for (int f = 0; f < 4; ++f) out[0][f] = p[f];
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
      out[j + 1][o] = p[o];
    }
  }
}

// Sum of x over the lanes 4i+f with equal f (i.e. over electrons, per unit f); every
// lane receives its class total.  row_ror:4, row_ror:8, then across the four rows.
template <typename T> __device__ __forceinline__ T class4_sum(T x) {
  x += dpp<0x124>(x);
  x += dpp<0x128>(x);
#ifdef AQ_PERMLANE_SUM
  if constexpr (sizeof(T) == 4) {
    // across the rows on the VALU (gfx950 row swaps; the same additions as the xor shuffles)
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
  }
#endif
  x += __shfl_xor(x, 16);
  x += __shfl_xor(x, 32);
  return x;
}
// Value of x held by lane M of this lane's quad.
template <int M, typename T> __device__ __forceinline__ T quad_bcast(T x) {
  return dpp<M | (M << 2) | (M << 4) | (M << 6)>(x);
}

// The first NU of an NV-element lane record (16-byte aligned) in loads of exactly those elements
// (16-, 8- and 4-byte; the rest set to zero): a 16-byte load whose unused elements' registers are
// reallocated must complete before they are overwritten, which placed a vmcnt(0) right behind the
// F4 weight prefetch
template <typename T, int NV, int NU>
__device__ __forceinline__ void ld_use(cptr<T> p, T* out) {
  static_assert(NU <= NV, "record");
  if constexpr (sizeof(T) == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    const __attribute__((address_space(4))) f4* q = (const __attribute__((address_space(4))) f4*)p;
#pragma unroll
    for (int j = 0; j < NU / 4; ++j) {
      const f4 v = q[j];
      out[4 * j] = v.x;
      out[4 * j + 1] = v.y;
      out[4 * j + 2] = v.z;
      out[4 * j + 3] = v.w;
    }
    constexpr int B = NU / 4 * 4, R = NU % 4;
    if constexpr (R >= 2) {
      const f2 v = *(const __attribute__((address_space(4))) f2*)(p + B);
      out[B] = v.x;
      out[B + 1] = v.y;
    }
    if constexpr (R == 1 || R == 3) out[B + R - 1] = p[B + R - 1];
#pragma unroll
    for (int k = NU; k < NV; ++k) out[k] = T(0);
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = k < NU ? p[k] : T(0);
  }
}

// NV (a multiple of 16 bytes' worth) consecutive parameters from a 16-byte aligned offset of the
// parameter buffer, in 16-byte loads (layout.h lane-order blocks)
template <typename T, int NV>
__device__ __forceinline__ void ld_vec(cptr<T> p, T* out) {
  if constexpr (sizeof(T) == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const __attribute__((address_space(4))) f4* q = (const __attribute__((address_space(4))) f4*)p;
#pragma unroll
    for (int j = 0; j < NV / 4; ++j) {
      const f4 v = q[j];
      out[4 * j] = v.x;
      out[4 * j + 1] = v.y;
      out[4 * j + 2] = v.z;
      out[4 * j + 3] = v.w;
    }
  } else {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const __attribute__((address_space(4))) d2* q = (const __attribute__((address_space(4))) d2*)p;
#pragma unroll
    for (int j = 0; j < NV / 2; ++j) {
      const d2 v = q[j];
      out[2 * j] = v.x;
      out[2 * j + 1] = v.y;
    }
  }
}
#ifndef AQ_NO_XLANE
constexpr bool kXLane = true;    // F4 / B2 read the lane-order weight blocks in 16-byte loads
#else
constexpr bool kXLane = false;
#endif

// Barrier of a one-configuration wave: LDS traffic of one wave is processed in order, so a
// wavefront-scope fence (a compiler barrier, no s_waitcnt) orders its cross-lane LDS accesses.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Kernel arguments read at the end of the kernel: through an opaque copy of the kernarg segment
// pointer, so that their loads are issued where they are used instead of being hoisted into SGPRs
// that live across the whole kernel (the proposal kernel spills SGPRs through VALU lane writes).
// The kernels take one argument (KArgs), at kernarg offset 0.
__device__ __forceinline__ const __attribute__((address_space(4))) KArgs* late_args() {
  auto p = (const __attribute__((address_space(4))) KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// Proposal B3's pair order (k, i) per moved electron pi and pair slot it = lane + 64 u: the
// 2(N-1) pairs of pi first (it < M), then the others in row-major order; slots past N(N-1)
// repeat the last pair.  Code = k | i << 4 | (k N + i) << 8 (the pair's walker-cache row).
template <int N> struct PairTab {
  static constexpr int M = 2 * (N - 1), NPR = N * (N - 1), NS = ((NPR + 63) / 64) * 64;
  unsigned short v[N][NS];
  constexpr PairTab() : v{} {
    for (int pi = 0; pi < N; ++pi)
      for (int it = 0; it < NS; ++it) {
        int k = 0, i = 0;
        if (it < M) {
          const int j = it < N - 1 ? it : it - (N - 1);
          const int o = j + (j >= pi ? 1 : 0);
          k = it < N - 1 ? pi : o;
          i = it < N - 1 ? o : pi;
        } else if (N > 2) {
          const int uu = (it < NPR ? it : NPR - 1) - M;
          const int kk = uu / (N - 2);
          const int jj = uu - kk * (N - 2);
          const int ii = jj + (jj >= kk ? 1 : 0);
          k = kk + (kk >= pi ? 1 : 0);
          i = ii + (ii >= pi ? 1 : 0);
        }
        v[pi][it] = (unsigned short)(k | (i << 4) | ((k * N + i) << 8));
      }
  }
};
template <int N> __constant__ PairTab<N> pair_tab{};

// n consecutive elements global -> LDS by gfx950 LDS-DMA (global_load_lds_dword: lane l of each
// wave-instruction writes the wave-uniform LDS base + 4 l; no VGPR destination).  The data is
// counted on vmcnt: the caller waits (s_waitcnt vmcnt(0)) before anything reads or overwrites it.
template <typename T>
__device__ __forceinline__ void lds_dma(T* dst, const T* src, int n, int lane) {
  const int nw = n * (int)sizeof(T) / 4;
  const float* s = (const float*)src;
  float* d = (float*)dst;
#pragma unroll
  for (int w = 0; w < nw; w += 64) {
    if (w + lane < nw)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(s + w + lane),
                                       (__attribute__((address_space(3))) void*)(d + w), 4, 0, 0);
  }
}

// c ? x : +0 as a bit mask (no select of a loaded value: see the F1 cache loads)
__device__ __forceinline__ float and_zero(bool c, float x) {
  return __builtin_bit_cast(float, __builtin_bit_cast(unsigned, x) & (c ? ~0u : 0u));
}
__device__ __forceinline__ double and_zero(bool c, double x) {
  return __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, x) & (c ? ~0ull : 0ull));
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2):
// give every XCD a contiguous range of configurations, so the N proposals of a
// walker (and that walker's cache) land on one L2.
__device__ __forceinline__ int xcd_major(int blk, int n) {
  if ((n & 7) != 0) return blk;
  return (blk & 7) * (n >> 3) + (blk >> 3);
}

// Electron-local stage of the moved electron of proposals q = 16*block + s (lane = 16c + s).
// The wave's 16 records are contiguous in the cache: they are assembled in LDS and written
// with coalesced stores (direct per-lane stores scatter over 16 records x 4 lanes).
// MOVED_WPB independent waves (16 proposals each) per workgroup: the launch pays per workgroup
// (see AQ_PROP_WPB); the grid is padded to a multiple of 8 and the padding waves exit.
// (round 4: 2 per workgroup, N2 iteration at 512 walkers 0.780-0.784 -> 0.770-0.777 ms, 4096 equal;
// 8: no better; profiles/r04_s9_ab_prop_wpb.txt)
#ifndef AQ_MOVED_WPB
#define AQ_MOVED_WPB 2
#endif
constexpr int MOVED_WPB = AQ_MOVED_WPB;
template <typename T, int N, int A>
__global__ __launch_bounds__(64 * MOVED_WPB) void k_moved_electron(KArgs ka) {
  using Ly = Lay<N, A>;
  using EC = ECache<N, A>;
  constexpr int D0 = 4 * A;
  // records padded by one element in LDS: EC::size is a multiple of 16, so an unpadded record
  // stride puts the 16 lanes of a direction row on one bank (16-way conflicts)
  constexpr int RS = EC::size + 1;
  __shared__ T ebw[MOVED_WPB][16 * RS];
  const cptr<T> P = param_ptr<T>(ka.prm);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  T* eb = ebw[wv];
  const int lane = threadIdx.x & 63;
  const int lc = lane >> 4, s = lane & 15;
  const int blk = xcd_major(blockIdx.x, gridDim.x) * MOVED_WPB + wv;
  if (blk * 16 >= ka.nconf) return;
  const int nrec = ka.nconf - blk * 16 < 16 ? ka.nconf - blk * 16 : 16;
  const int q = blk * 16 + (s < nrec ? s : nrec - 1);
  const int mper = ka.mper ? ka.mper : N, mdiv = ka.mdiv ? ka.mdiv : 1;
  const int b = q / mper, i = (q - b * mper) / mdiv;
  T xp[3];
  if (ka.xnew) {
#pragma unroll
    for (int c = 0; c < 3; ++c) xp[c] = ((const T*)ka.xnew)[(size_t)q * 3 + c];
  } else {
    const T tstep = (T)ka.tstep;
    const T te = taueff_wave<T>(ka.taueff, ka.tacc, 0, ka.tstep, ka.tpart);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o = (size_t)b * 3 * N + 3 * i + c;
      const T ge = ((const T*)ka.pgrad)[o] * te;
      xp[c] = ((const T*)ka.pos)[o] + (ge * tstep + f_sqrt(tstep) * ((const T*)ka.gauss1)[o]);
    }
  }
  ElecOut<T, A> eo;
  electron_stage<T, N, A>(P, xp, i, lc, eo);
  T* E = eb + s * RS;
#pragma unroll
  for (int col = 0; col < N; ++col) {
    PJ<T> sy = P[Ly::wy + col] * eo.yst[0];
#pragma unroll
    for (int m = 1; m < NYW; ++m) sy = sy + P[Ly::wy + m * N + col] * eo.yst[m];
    const PJ<T> yt = eo.env * sy;
    if (lc == 3) E[EC::yv + col] = yt.v;
    else E[EC::yd + lc * N + col] = yt.d1;
  }
#pragma unroll
  for (int m = 0; m < D0; ++m) {
    if (lc == 3) E[EC::h0 + m] = eo.hf[m].v;
    else E[EC::hd + lc * D0 + m] = eo.hf[m].d1;
  }
  if (lc == 3) E[EC::jv] = eo.jae.v;
  else E[EC::jd + lc] = eo.jae.d1;
  if (lc == 3) {
#pragma unroll
    for (int c = 0; c < 3; ++c) E[EC::xp + c] = xp[c];
  }
  wave_sync();   // the wave's own records (waves of a workgroup share nothing)
  T* dst = (T*)ka.ecache + (size_t)blk * 16 * EC::size;
  for (int idx = lane; idx < nrec * EC::size; idx += 64) {
    const int rec = idx / EC::size;
    dst[idx] = eb[idx + rec];
  }
}

// Value-only records for the pp quadrature configurations (ka.value_only): their consumers
// (k_quad_value, the value-only proposal path) read the Yt row, the ae features, J_ae and the
// position only, so one configuration per lane (the value row of electron_stage) instead of one
// per 16-lane direction row: a quarter of the waves.
template <typename T, int N, int A>
__global__ __launch_bounds__(64 * MOVED_WPB) void k_moved_value(KArgs ka) {
  using Ly = Lay<N, A>;
  using EC = ECache<N, A>;
  constexpr int D0 = 4 * A;
  const cptr<T> P = param_ptr<T>(ka.prm);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int q0 = (xcd_major(blockIdx.x, gridDim.x) * MOVED_WPB + wv) * 64 + lane;
  if (q0 >= ka.nconf) return;
  const int mper = ka.mper ? ka.mper : N, mdiv = ka.mdiv ? ka.mdiv : 1;
  const int b = q0 / mper, i = (q0 - b * mper) / mdiv;
  T xp[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) xp[c] = ((const T*)ka.xnew)[(size_t)q0 * 3 + c];
  ElecOut<T, A> eo;
  electron_stage<T, N, A>(P, xp, i, 3, eo);
  T* E = (T*)ka.ecache + (size_t)q0 * EC::size;
#pragma unroll
  for (int col = 0; col < N; ++col) {
    PJ<T> sy = P[Ly::wy + col] * eo.yst[0];
#pragma unroll
    for (int m = 1; m < NYW; ++m) sy = sy + P[Ly::wy + m * N + col] * eo.yst[m];
    E[EC::yv + col] = (eo.env * sy).v;
  }
#pragma unroll
  for (int m = 0; m < D0; ++m) E[EC::h0 + m] = eo.hf[m].v;
  E[EC::jv] = eo.jae.v;
#pragma unroll
  for (int c = 0; c < 3; ++c) E[EC::xp + c] = xp[c];
}

// Occupancy hint per instantiation: fp32 N2 (14, 2) lands one VGPR above the
// 4-waves/SIMD budget (128) without it and fits it without spilling with it.
// PREP (the adjoint pass of the local energy, walker_lap.h) asks for 2.
#ifndef AQ_PROP_WAVES
#define AQ_PROP_WAVES 5
#endif
#ifndef AQ_PREP_WAVES
#define AQ_PREP_WAVES 4
#endif
template <typename T, int N, int A, bool PREP, bool PROP, bool PW7 = false> struct RevWaves {
  static constexpr int value = PW7 ? 7 : (PREP ? (sizeof(T) == 4 ? AQ_PREP_WAVES : 2) : ((sizeof(T) == 4 && N == 14 && A == 2) ? (PROP ? AQ_PROP_WAVES : 4) : 1));
};

// PREP = false: value + gradient (Metropolis walker launches and single-electron proposal / ECP
//   quadrature launches; ka.proposal selects the path at run time).  PROP only selects the
//   occupancy target of the instantiation: fp32 N2 proposals fit 5 waves/SIMD (90 VGPRs, 8.1 KB
//   LDS), the walker launch (4096 waves, one round) is faster compiled for 4.  Making the path a
//   compile-time choice was measured worse: the proposal-only code spilled at the 5-wave budget.
// PREP = true : first launch of the local energy (walker_lap.h): values, the adjoint pass
//   through the h stream, and the pair stream's derivative sums and curvature, written to
//   the walker's LapCache; no gradient (B3/B4) and no Metropolis cache.
// Proposal launches: AQ_PROP_WPB configurations (one wave each) per workgroup; the waves share
// nothing, so their LDS regions are disjoint and every barrier is wave-local.
// (round 4, re-measured on the final code: 2 per workgroup beats 4 at 4096 N2 walkers, proposal
// launch 222.3-224.9 -> 219.1-222.0 us, iteration 2.990-3.019 -> 2.962-2.997 ms; 1 and 8 are slower,
// 512 walkers equal; profiles/r04_s9_ab_prop_wpb.txt)
#ifndef AQ_PROP_WPB
#define AQ_PROP_WPB 2
#endif
#ifndef AQ_WALK_WPB
#define AQ_WALK_WPB 1
#endif
template <typename T, bool PROP, bool PREP = false> struct RevWpb {
  static constexpr int value = sizeof(T) != 4 ? 1 : (PROP ? AQ_PROP_WPB : (PREP ? 1 : AQ_WALK_WPB));
};
#ifdef AQ_WAVE_SYNC
#define AQ_SYNC() wave_sync()
#else
#define AQ_SYNC()                                   \
  do {                                              \
    if constexpr (WPB > 1) wave_sync();             \
    else __syncthreads();                           \
  } while (0)
#endif

// One ordered pair (k, i) of B3 (walker_rev's pair adjoints): forward values (fresh) or the cached
// t1, t2, then the adjoints back through the two double layers to d = x_i - x_k, into dbar
// (a function so that both waves of a split walker launch can run it on their share of the pairs).
// may_fresh (compile-time after unrolling): the pair may recompute its forward values; fresh
// selects them per lane without a branch (a divergent branch here turned the uniform weights
// into per-lane copies at the merge)
template <typename T, int N, int A>
__device__ __forceinline__ void b3_pair_adjoint(cptr<T> P, const T* xs, const T* g2b, T* dbar, int nup, int k, int i,
                                                bool may_fresh, bool fresh, const T* tcache, T cusp, T al) {
  using Ly = Lay<N, A>;
  const T RSQ2 = T(0.70710678118654752);
  // the uniform layer weights are re-read per pair from the scalar cache (s_load) instead of
  // being kept in SGPRs across the kernel (which spills them through VALU lane writes)
  cptr<T> Pq = P;
  asm volatile("" : "+s"(Pq));
  const int G = k >= nup ? 1 : 0;
  T d[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) d[c] = xs[i * 3 + c] - xs[k * 3 + c];
  const T r = f_sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  T p0[4] = {r, d[0], d[1], d[2]};
  T t1[4], t2[4];
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    t1[o] = tcache ? tcache[o] : T(0);
    t2[o] = tcache ? tcache[4 + o] : T(0);
  }
  if (may_fresh) {
    // recompute the two double layers (values)
    T f1[4], p1[4], f2[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      T s = Pq[Ly::dbl_b0 + o];
#pragma unroll
      for (int m = 0; m < 4; ++m) s += p0[m] * Pq[Ly::dbl_w0 + m * 4 + o];
      f1[o] = f_tanh(s);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) p1[o] = (p0[o] + f1[o]) * RSQ2;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      T s = Pq[Ly::dbl_b1 + o];
#pragma unroll
      for (int m = 0; m < 4; ++m) s += p1[m] * Pq[Ly::dbl_w1 + m * 4 + o];
      f2[o] = f_tanh(s);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      t1[o] = fresh ? f1[o] : t1[o];
      t2[o] = fresh ? f2[o] : t2[o];
    }
  }
  // adjoints: output of layer l feeds g2[l][G][i] with weight 1/|G|
  T pb2[4], pb1[4], pb0[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) pb2[f] = g2b[((2 * 2 + G) * N + i) * 4 + f];
  T z2[4];
#pragma unroll
  for (int o = 0; o < 4; ++o) z2[o] = pb2[o] * RSQ2 * (T(1) - t2[o] * t2[o]);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    T s = g2b[((1 * 2 + G) * N + i) * 4 + m] + pb2[m] * RSQ2;
#pragma unroll
    for (int o = 0; o < 4; ++o) s += z2[o] * Pq[Ly::dbl_w1 + m * 4 + o];
    pb1[m] = s;
  }
  T z1[4];
#pragma unroll
  for (int o = 0; o < 4; ++o) z1[o] = pb1[o] * RSQ2 * (T(1) - t1[o] * t1[o]);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    T s = g2b[((0 * 2 + G) * N + i) * 4 + m] + pb1[m] * RSQ2;
#pragma unroll
    for (int o = 0; o < 4; ++o) s += z1[o] * Pq[Ly::dbl_w0 + m * 4 + o];
    pb0[m] = s;
  }
  // p0 = [r, d]; Pade e-e Jastrow once per unordered pair (k < i)
  T rb = pb0[0];
  {
    // the pair's Jastrow parameters come loaded on every lane and are masked here (a branch
    // around their loads waited for every load in flight, the cached tanh's included)
    const T den = al * r + T(1);
    rb += and_zero(k < i, cusp * f_rcp(den * den));
  }
  const T ir = f_rcp(r);
#pragma unroll
  for (int c = 0; c < 3; ++c) dbar[(k * N + i) * 3 + c] = pb0[1 + c] + rb * d[c] * ir;
}

// The sweep's draws of walker conf (k_draws' arithmetic, fused into the walker launch)
template <typename T, int N>
__device__ __forceinline__ void walker_draws(const __attribute__((address_space(4))) KArgs* kl, int conf, int lane) {
  if (kl->dg1 && lane < N) {
    const uint32_t t = (uint32_t)(conf * N + lane);
    const uint64_t seed = kl->seed, step = kl->step;
    float a[3], b[3], c[4];
    philox_normal3f(seed, step, t, 0u, a);
    philox_normal3f(seed, step, t, 1u, b);
    philox_u4(seed, step, t, 2u, c);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ((T*)kl->dg1)[(size_t)t * 3 + k] = (T)a[k];
      ((T*)kl->dg2)[(size_t)t * 3 + k] = (T)b[k];
    }
    ((T*)kl->du)[t] = (T)(c[0] - 5.9604644775390625e-08f);
  }
}

// PW7 (proposals only, -DAQ_PW7 builds: measured slower, shape.hip): the small-batch instantiation, compiled for 7 waves/SIMD with the COMPACT
// LDS layout, so that the B N proposals of a strong-scaling rank (512 N2 walkers: 7,168 waves) run
// in one round instead of 1.4 (shape.hip chooses it by batch size)
// PH (PREP only): the adjoint pass of the PHASE -- seeded by Im d log det / dH instead of Re, so
// that the LapCache's node weights, feature adjoints and pair-local curvature are those of
// theta = arg psi (the complex_output=True kinetic energy, hamiltonian.py:110-130)
// SPL (walker launches of small batches, shape.hip): two waves per walker -- wave 0 the
// per-electron stage F1 and everything after F2, wave 1 the pair stream F2 (its walker-cache rows,
// the column sums g2, J_ee) at the same time; wave 1 hands g2 and J_ee over through LDS at one
// workgroup barrier and exits.  F1 and F2 depend on the positions only (nn.py:106-153).
template <typename T, int N, int A, bool PREP = false, bool PROP = false, bool PW7 = false, bool PH = false,
          bool SPL = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 64 * (SPL ? 2 : RevWpb<T, PROP, PREP>::value)))) __attribute__((amdgpu_waves_per_eu(RevWaves<T, N, A, PREP, PROP, PW7>::value))) void
k_walker_rev(KArgs ka) {
  static_assert(!PW7 || (PROP && !PREP), "PW7 is a proposal instantiation");
  static_assert(!PH || PREP, "PH is an adjoint-pass instantiation");
  static_assert(!SPL || (!PROP && !PREP), "SPL is a walker-launch instantiation");
  using Ly = Lay<N, A>;
  constexpr bool fwd_reg = PROP && kFwdReg;
  constexpr bool compact = PROP && PW7 && fwd_reg;
  // the lane-order weight blocks in F4 / B2: proposals only (round 4, interleaved A/B on one box:
  // proposal launch 216.3-219.0 -> 215.1-218.2 us; the same in the walker launch and the local
  // energy's adjoint pass measured +0.5 us and +7-11 us per launch, profiles/r04_s5_ab_xlane.txt)
  constexpr bool xlane = PROP && kXLane;
  using SM = SmemRev<T, N, A, fwd_reg, compact>;
  using LCc = LapCache<N, A>;
  constexpr int D0 = SM::D0;
  constexpr int WPB = SPL ? 2 : RevWpb<T, PROP, PREP>::value;
  const cptr<T> P = param_ptr<T>(ka.prm);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  // wave index within the workgroup, wave-uniform (scalar)
  const int wv = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  // SPL: both waves work on one walker's LDS block
  T* sm = (T*)(smem_raw + (SPL ? 0 : wv) * SM::bytes);
  T* xs = sm + SM::xs;

  // The PROP instantiation is launched only for proposals that read the walker cache (shape.hip
  // routes reuse-off proposals to the general one), so there both path flags are compile-time.
  const bool isprop = PROP ? true : (ka.proposal != 0);
  const int conf = SPL ? xcd_major(blockIdx.x, gridDim.x) : xcd_major(blockIdx.x, gridDim.x) * WPB + wv;
  if (WPB > 1 && conf >= ka.nconf) return;
  const int lane = WPB > 1 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  const int lc = lane >> 4;
  const int er = lane & 15;
  const int le = er < N ? er : N - 1;
  const bool val = (lc == 3);
  const bool live = er < N;
  const bool dir = (lc < 3) && live;
  const int nup = ka.nup;
  const T tstep = (T)ka.tstep;
  const T RSQ2 = T(0.70710678118654752);
  const T ginv0 = T(1) / T(nup), ginv1 = T(1) / T(N - nup);
  const int* rowsrc = ka.rowsrc;
#ifdef AQ_PHASE_PROF
  unsigned long long t_ph = __builtin_readcyclecounter();
#endif

  // ------------------------------------------------------------------ F0 positions (as k_walker)
  int pb = conf, pi = -1;
  if (isprop) {
    const int mper = ka.mper ? ka.mper : N, mdiv = ka.mdiv ? ka.mdiv : 1;
    pb = conf / mper;
    pi = (conf - pb * mper) / mdiv;
  }
  // reuse-off proposals: the walker limdrift factor, read by the wave before the divergent F0
  const T te_walk = (!PROP && isprop && !ka.xnew) ? taueff_wave<T>(ka.taueff, ka.tacc, 0, ka.tstep, ka.tpart) : T(0);
  if (SPL && wv != 0) {
    // SPL wave 1: the positions come from wave 0 (after its acceptance) through LDS
  } else if (!PREP && !isprop && ka.acc.lpn) {
    // the previous sweep's acceptance of this walker's N proposals (k_accept's arithmetic)
    const T te1 = taueff_wave<T>(ka.acc.taueff, ka.acc.tacc, 0, ka.acc.tstep, ka.acc.tpart);
    const T te2 = taueff_wave<T>(ka.acc.taueff, ka.acc.tacc, 1, ka.acc.tstep, ka.acc.tpart);
    if (lane < N) {
      T xn[3];
      const bool acc = accept_one<T, N>(ka.acc, (const T*)ka.pos, conf, lane, xn, te1, te2);
#pragma unroll
      for (int c = 0; c < 3; ++c) xs[3 * lane + c] = xn[c];
      if (acc) {
#pragma unroll
        for (int c = 0; c < 3; ++c) ((T*)ka.pos)[(size_t)conf * 3 * N + 3 * lane + c] = xn[c];
        if (ka.acc.count) atomicAdd(&ka.acc.count[conf], 1);
      }
    }
  } else if (!PROP && lane < 3 * N) {   // PROP: positions come with the cache loads of F1
    T x = ((const T*)ka.pos)[(size_t)pb * 3 * N + lane];
    if (isprop && lane / 3 == pi) {
      sm[SM::R + (lane - 3 * pi)] = x;                       // old position of the moved electron
      if (ka.xnew) {
        x = ((const T*)ka.xnew)[(size_t)conf * 3 + (lane - 3 * pi)];
      } else {
        const T z = ((const T*)ka.gauss1)[(size_t)pb * 3 * N + lane];   // drawn by the host or k_draws
        const T ge = ((const T*)ka.pgrad)[(size_t)pb * 3 * N + lane] * te_walk;
        x = x + (ge * tstep + f_sqrt(tstep) * z);
      }
    }
    xs[lane] = x;
  }
  if constexpr (SPL) __syncthreads();   // wave 1 reads the positions
  else if constexpr (!PROP) AQ_SYNC();

  AQ_PH(0);
  // ------------------------------------------------------------------ F1 per-electron stage (electron.h)
  // Walker cache: read (proposal with reuse: this proposal's walker pb) or written (by conf).
  using WC = WCache<N, A>;
  using EC = ECache<N, A>;
  // shape.hip launches every proposal that reads the walker cache with the PROP instantiation, so
  // the cached path is compiled there only (the general one serves walker launches, reuse-off
  // proposals and plain value+gradient calls)
  const bool reuse = !PREP && PROP;
  // PROP: F1's walker-cache blocks by LDS-DMA (round 6, interleaved A/B on one box, N2 4096 walkers,
  // µs per proposal launch: 220.7 / 221.4 -> 220.5 / 220.6, positions bitwise equal; 21 VALU and one
  // VGPR fewer per wave; profiles/r06_s1_ab_f1_glds_slp.txt).  -DAQ_NO_F1_GLDS: VGPR-staged copies.
#ifndef AQ_NO_F1_GLDS
  constexpr bool f1_glds = PROP;
#else
  constexpr bool f1_glds = false;
#endif
  // walker launch re-using its previous sweep's pivot order (F5; KArgs::pvok)
  const bool wfix = !PREP && !PROP && !isprop && ka.pvok != 0;
  T* Wc = (T*)ka.wcache + (size_t)(reuse ? pb : conf) * WC::size;
  T* Lw = PREP ? (T*)ka.lapcache + (size_t)conf * LCc::size : nullptr;
  const T* Eq = reuse ? (const T*)ka.ecache + (size_t)conf * EC::size : nullptr;
  T* Yv = sm + SM::yv;
  T* g2 = sm + SM::g2;
  T jv = T(0), jd1 = T(0), jve = T(0);
  T jsum_p = T(0);   // fwd_reg: wave_sum(jv + jve), formed in F2
  T pvr = T(0);
  int rsl = 0;   // PROP: rowsrc[lane]
  T jvp = T(0);  // F2's Jastrow terms of the moved electron's pairs
  // F2 of a proposal, first half: the 2(N-1) pairs of the moved electron pi, lane = 16 part + o:
  // part 0/1: pair (pi, o) at the new/old x_pi (column o); part 2/3: pair (o, pi) (column pi);
  // their stream values to S [64][12], the e-e Jastrow change to jvp
  auto f2_pair_values = [&](T cusp, T al) {   // PROP: the pair's Jastrow parameters, loaded early
    T* S = sm + SM::R + 4;
    const T* xo = sm + SM::R;                       // old position of pi
    const int o = lane & 15, part = lane >> 4;
    const int os = o < N ? o : N - 1;
    const T* xp = (part & 1) ? xo : xs + pi * 3;
    T d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = (part < 2) ? xs[os * 3 + c] - xp[c] : xp[c] - xs[os * 3 + c];
    T v[3][4];
    pair_values<T, N, A>(d, P, v);
    if constexpr (compact) {
      // new - old: part 1 (3) sends its values to part 0 (2) sixteen lanes down; D[16 (part / 2) + o]
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const T w = __shfl_down(v[l][f], 16);
          if ((part & 1) == 0) S[(16 * (part >> 1) + o) * 12 + l * 4 + f] = v[l][f] - w;
        }
    } else {
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
      for (int f = 0; f < 4; ++f) S[lane * 12 + l * 4 + f] = v[l][f];
    }
    if (part < 2 && o < N && o != pi) {
      if constexpr (!PROP) {
        cusp = P[Ly::jee_c + pi * N + o];
        al = P[Ly::jee_a + pi * N + o];
      }
      const T je = f_div(cusp * v[0][0], al * v[0][0] + T(1));
      jvp += part == 0 ? je : -je;
    }
  };
  // the Jastrow parameters of pair (pi, o) of this lane (o = lane & 15, clamped)
  auto jee_params = [&](T& cusp, T& al) {
    const int os = (lane & 15) < N ? (lane & 15) : N - 1;
    cusp = P[Ly::jee_c + pi * N + os];
    al = P[Ly::jee_a + pi * N + os];
  };
  if (reuse) {
    // walker pb's cached stage and pair sums, electron pi's entries from k_moved_electron;
    // all loads issued before the first LDS store
    constexpr int NY = (N * N + 63) / 64, NHh = (N * D0 + 63) / 64, NG = (3 * 2 * N * 4 + 63) / 64;
    T ry[NY], rh[NHh], rg[NG];
    // f1_glds: the walker's Yt, ae-feature and g2 blocks go global -> LDS by LDS-DMA (no VGPR
    // staging, no per-element selection); the moved electron's rows are patched in after they land
    T eyv = T(0), eh0 = T(0);
    if constexpr (f1_glds) {
      lds_dma<T>(Yv, Wc + WC::yv, N * N, lane);
      lds_dma<T>(sm + SM::hl, Wc + WC::h0, N * D0, lane);
      lds_dma<T>(g2, Wc + WC::g2, 3 * 2 * N * 4, lane);
      eyv = Eq[EC::yv + (lane < N ? lane : N - 1)];
      eh0 = Eq[EC::h0 + (lane < D0 ? lane : D0 - 1)];
    }
    // PROP: F0's positions too (walker pb's, the moved electron's proposed position from
    // k_moved_electron), so that every global load of F0/F1 is in flight before one barrier
    // Every load is issued unconditionally at a clamped, in-bounds index and the moved electron's
    // entries are selected afterwards: no divergent branch (exec-mask save/restore) per element.
    const bool mvl = lane < 3 * N && lane / 3 == pi;
    T x0 = T(0), xm = T(0), jc = T(0), ja = T(0);
    if constexpr (PROP) {
      const int l3 = lane < 3 * N ? lane : 3 * N - 1;
      x0 = ((const T*)ka.pos)[(size_t)pb * 3 * N + l3];
      xm = Eq[EC::xp + (mvl ? lane - 3 * pi : 0)];
      jee_params(jc, ja);   // before the cache loads: F2's pair values wait for these only
      rsl = rowsrc[lane < N ? lane : N - 1];   // F5's slot table (after F4)
    }
    // unsigned offsets: the loads take the wave's base pointer in SGPRs plus a 32-bit lane offset
    if constexpr (!f1_glds) {
#pragma unroll
    for (int t = 0; t < NY; ++t) {
      const unsigned idx = lane + 64 * t;
      const unsigned ix = idx < N * N ? idx : N * N - 1;
      const unsigned r = ix / N;
      const T a = Wc[WC::yv + ix], b = Eq[EC::yv + (ix - r * N)];
      ry[t] = ((int)r == pi) ? b : a;
    }
#pragma unroll
    for (int t = 0; t < NHh; ++t) {
      const unsigned idx = lane + 64 * t;
      const unsigned ix = idx < N * D0 ? idx : N * D0 - 1;
      const unsigned e = ix / D0;
      const T a = Wc[WC::h0 + ix], b = Eq[EC::h0 + (ix - e * D0)];
      rh[t] = ((int)e == pi) ? b : a;
    }
#pragma unroll
    for (int t = 0; t < NG; ++t) {
      const int idx = lane + 64 * t;
      rg[t] = Wc[WC::g2 + (idx < 3 * 2 * N * 4 ? idx : 3 * 2 * N * 4 - 1)];
    }
    }
    {
      // one load per value from a selected address, masked to +0 by a bit and: a select between
      // two loaded values (or a loaded value and 0) is turned into a branch around the loads by
      // the compiler, and the branch waits for every load issued so far
      if constexpr (PROP) {
        const T* js = (er == pi) ? Eq + EC::jv : Wc + WC::jaev + le;
        jv = and_zero(val && live, *js);
        const T* ds = (le == pi) ? Eq + EC::jd + (lc < 3 ? lc : 0) : Wc + WC::jaed + (lane < 48 ? lane : 47);
        jd1 = and_zero(dir, *ds);
        jve = and_zero(lane == 0, Wc[WC::jee]);
      } else {
        const T a = Wc[WC::jaev + le], b = Eq[EC::jv];
        jv = (val && live) ? ((er == pi) ? b : a) : T(0);
        const T a1 = Wc[WC::jaed + (lane < 48 ? lane : 47)], b1 = Eq[EC::jd + (lc < 3 ? lc : 0)];
        jd1 = dir ? ((le == pi) ? b1 : a1) : T(0);
        const T a2 = Wc[WC::jee];
        jve = lane == 0 ? a2 : T(0);
      }
      pvr = Wc[WC::pv + (lane < 2 * N + 2 ? lane : 2 * N + 1)];   // to LDS after F4 (SmemRev::pv)
    }
    if constexpr (PROP) {
      if (mvl) sm[SM::R + (lane - 3 * pi)] = x0;             // old position of the moved electron
      if (lane < 3 * N) xs[lane] = mvl ? xm : x0;
      // F2's pair values of the moved electron need the positions only: computed while the
      // cache loads above are still in flight (they are waited for at the LDS stores below)
      AQ_SYNC();
      f2_pair_values(jc, ja);
    }
    if constexpr (f1_glds) {
      // the DMA'd blocks have landed (vmcnt counts LDS-DMA) before the moved electron's rows go over them
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < N) Yv[pi * N + lane] = eyv;
      if (lane < D0) sm[SM::hl + pi * D0 + lane] = eh0;
    } else {
#pragma unroll
    for (int t = 0; t < NY; ++t)
      if (lane + 64 * t < N * N) Yv[lane + 64 * t] = ry[t];
#pragma unroll
    for (int t = 0; t < NHh; ++t)
      if (lane + 64 * t < N * D0) sm[SM::hl + lane + 64 * t] = rh[t];
#pragma unroll
    for (int t = 0; t < NG; ++t)
      if (lane + 64 * t < 3 * 2 * N * 4) g2[lane + 64 * t] = rg[t];
    }
  } else if (!SPL || wv == 0) {
    if (wfix) pvr = Wc[WC::pv + (lane < 3 * N + 2 ? lane : 3 * N + 1)];   // to LDS after F4, before F5's write
    ElecOut<T, A> eo;
    electron_stage<T, N, A>(P, xs + le * 3, le, lc, eo);
    // d(Yt row)/dx and d(ae features)/dx of this lane's electron -> walker cache (read in B4)
    T* Wl = Wc + WC::loc + lane;
#pragma unroll
    for (int col = 0; col < N; ++col) {
      PJ<T> sy = P[Ly::wy + col] * eo.yst[0];
#pragma unroll
      for (int m = 1; m < NYW; ++m) sy = sy + P[Ly::wy + m * N + col] * eo.yst[m];
      const PJ<T> yt = eo.env * sy;
      if (!PREP && lane < 48) Wl[col * 48] = yt.d1;
      if (val && live) Yv[er * N + col] = yt.v;
    }
#pragma unroll
    for (int m = 0; m < D0; ++m) {
      if (!PREP && lane < 48) Wl[(N + m) * 48] = eo.hf[m].d1;
      if (val && live) sm[SM::hl + er * D0 + m] = eo.hf[m].v;
    }
    jv = (val && live) ? eo.jae.v : T(0);
    jd1 = dir ? eo.jae.d1 : T(0);
    if (!PREP && !isprop) {
      if (val && live) Wc[WC::jaev + er] = eo.jae.v;
      if (lane < 48) Wc[WC::jaed + lane] = jd1;
    }
  }
  AQ_SYNC();
  if (!PREP && !isprop && (!SPL || wv == 0)) {
    for (int idx = lane; idx < N * N; idx += 64) Wc[WC::yv + idx] = Yv[idx];
    for (int idx = lane; idx < N * D0; idx += 64) Wc[WC::h0 + idx] = sm[SM::hl + idx];
  }

  AQ_PH(1);
  // ------------------------------------------------------------------ F2+F3 pair stream + spin-group column means
  // lane = (column i, quarter kq): pairs (k, i) with k = kq, kq+4, ...; the three layers'
  // h2[k,i] values are summed per spin group in registers and quad-reduced with DPP.
  if (reuse && !AQ_ABL(1)) {
    // patch walker pb's sums with the 2(N-1) pairs of the moved electron pi. lane = 16*part + o:
    // part 0/1: pair (pi, o) at the new/old x_pi (column o); part 2/3: pair (o, pi) (column pi)
    T* S = sm + SM::R + 4;                          // [64][12] pair-stream values
    if constexpr (!PROP) {                          // PROP: done during the cache loads (F1)
      f2_pair_values(T(0), T(0));
      AQ_SYNC();
    }
    jve += jvp;
    if constexpr (fwd_reg) {
      // the Jastrow terms are complete: their wave sum (log|psi| = logdet + it) and the e-n
      // gradient of the direction lanes (B4) leave the registers until the end of the kernel
      jsum_p = wave_sum(jv + jve);
      sm[SM::jdo + lane] = jd1;
      jv = jve = jd1 = T(0);
    }
    if (lane < 16) {
      if (lane < N && lane != pi) {
        const int Gp = pi >= nup ? 1 : 0;
        const T gw = Gp ? ginv1 : ginv0;
#pragma unroll
        for (int l = 0; l < 3; ++l)
#pragma unroll
          for (int f = 0; f < 4; ++f)
            g2[((l * 2 + Gp) * N + lane) * 4 + f] +=
                (compact ? S[lane * 12 + l * 4 + f] : S[lane * 12 + l * 4 + f] - S[(16 + lane) * 12 + l * 4 + f]) * gw;
      }
    } else if (lane < 40) {
      const int t = lane - 16;
      const int l = t >> 3, G = (t >> 2) & 1, f = t & 3;
      const int k0 = G ? nup : 0, k1 = G ? N : nup;
      T acc = T(0);
      // unrolled over every k with the group and pi masked out (+0), so that the LDS reads are
      // issued together instead of one dependent round trip per electron of the group
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const T dv = compact ? S[(16 + k) * 12 + l * 4 + f] : S[(32 + k) * 12 + l * 4 + f] - S[(48 + k) * 12 + l * 4 + f];
        acc += (k >= k0 && k < k1 && k != pi) ? dv : T(0);
      }
      g2[((l * 2 + G) * N + pi) * 4 + f] += acc * (G ? ginv1 : ginv0);
    }
  } else if (!reuse && (!SPL || wv == 1)) {
    {
      const int i = lane >> 2, kq = lane & 3;
      const bool icol = i < N;
      const int ii = icol ? i : N - 1;
      T acc[3][2][4];
  #pragma unroll
      for (int l = 0; l < 3; ++l)
  #pragma unroll
        for (int G = 0; G < 2; ++G)
  #pragma unroll
          for (int f = 0; f < 4; ++f) acc[l][G][f] = T(0);
      // the e-e Jastrow parameters of the lane's pairs, all issued before the first pair (loaded in the
      // pair loop's k < i branch, each was a global round trip waited for on its own)
      constexpr int NT = (N + 3) / 4;
      T jcp[NT], jap[NT];
  #pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int kk = kq + 4 * t < N ? kq + 4 * t : N - 1;
        jcp[t] = P[Ly::jee_c + kk * N + ii];
        jap[t] = P[Ly::jee_a + kk * N + ii];
      }
      // the two double layers' weights, loaded once before the pair loop (element loads: their offsets
      // are not 16-byte aligned for every shape; the compiler merges them into wide scalar loads).  Read
      // inside the loop they were re-issued and waited for per pair
      T dwv[2][16], dbv[2][4];
  #pragma unroll
      for (int j = 0; j < 2; ++j) {
        const cptr<T> dw = P + (j == 0 ? Ly::dbl_w0 : Ly::dbl_w1);
        const cptr<T> db = P + (j == 0 ? Ly::dbl_b0 : Ly::dbl_b1);
  #pragma unroll
        for (int k = 0; k < 16; ++k) dwv[j][k] = dw[k];
  #pragma unroll
        for (int k = 0; k < 4; ++k) dbv[j][k] = db[k];
      }
  #pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int k = kq + 4 * t;
        if (k < N) {
          const bool diag = (k == ii);
          T d[3];
  #pragma unroll
          for (int c = 0; c < 3; ++c) d[c] = xs[ii * 3 + c] - xs[k * 3 + c];
          const T r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
          const T r = f_sqrt(diag ? T(1) : r2);
          T p[4] = {diag ? T(0) : r, diag ? T(0) : d[0], diag ? T(0) : d[1], diag ? T(0) : d[2]};
          if (icol && k < ii) {
            const T cusp = jcp[t], al = jap[t];
            jve += f_div(cusp * r, al * r + T(1));
          }
          const bool G1 = k >= nup;
  #pragma unroll
          for (int f = 0; f < 4; ++f) {
            acc[0][0][f] += G1 ? T(0) : p[f];
            acc[0][1][f] += G1 ? p[f] : T(0);
          }
  #pragma unroll
          for (int j = 0; j < 2; ++j) {
            T q[4];
  #pragma unroll
            for (int o = 0; o < 4; ++o) {
              T s = dbv[j][o];
  #pragma unroll
              for (int m = 0; m < 4; ++m) s += p[m] * dwv[j][m * 4 + o];
              q[o] = f_tanh(s);
            }
            if (!PREP && !isprop && icol && !diag) {   // walker cache: t_{j+1} of pair (k, i)
              T* tp = Wc + WC::pt + (k * N + ii) * 8 + j * 4;
#pragma unroll
              for (int o = 0; o < 4; ++o) tp[o] = q[o];
            }
            if (PREP && icol) {   // LapCache: the same for k_walker_lap, the diagonal's finite values included
              T* tp = Lw + LCc::pt + (k * N + ii) * LCc::pt_n + j * 4;
#pragma unroll
              for (int o = 0; o < 4; ++o) tp[o] = q[o];
            }
  #pragma unroll
            for (int o = 0; o < 4; ++o) {
              p[o] = (p[o] + q[o]) * RSQ2;
              acc[j + 1][0][o] += G1 ? T(0) : p[o];
              acc[j + 1][1][o] += G1 ? p[o] : T(0);
            }
          }
        }
      }
  #pragma unroll
      for (int l = 0; l < 3; ++l)
  #pragma unroll
        for (int G = 0; G < 2; ++G)
  #pragma unroll
          for (int f = 0; f < 4; ++f) {
            T v = acc[l][G][f];
            v += dpp<0xB1>(v);
            v += dpp<0x4E>(v);
            if (icol && kq == 0) g2[((l * 2 + G) * N + i) * 4 + f] = v * (G ? ginv1 : ginv0);
          }
    }
  }
  AQ_SYNC();
  if (!PREP && !isprop && (!SPL || wv == 1)) {
    for (int idx = lane; idx < 3 * 2 * N * 4; idx += 64) Wc[WC::g2 + idx] = g2[idx];
    const T je = wave_sum(jve);
    if (lane == 0) Wc[WC::jee] = je;
    if (SPL) sm[SM::R + lane] = jve;   // per lane, so that wave 0's sums keep their order (region R is free until F5)
  }
  if constexpr (SPL) {
    __syncthreads();   // wave 0 has the stage (F1), wave 1 the pair sums g2 and J_ee (F2)
    if (wv != 0) {
      // wave 1: the sweep's draws of this walker, then its half of B3 once wave 0 has the
      // adjoints g2b (B2) -- the pairs it = 64 + lane, 192 + lane, ... (wave 0 takes the others)
      walker_draws<T, N>(late_args(), conf, lane);
      if (ka.wcache) {
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        constexpr int NPR = N * (N - 1);
        for (int it = 64 + lane; it < NPR; it += 128) {
          const int k = it / (N - 1);
          const int jj = it - k * (N - 1);
          const int i = jj + (jj >= k ? 1 : 0);
          b3_pair_adjoint<T, N, A>(P, xs, sm + SM::g2, sm + SM::dbar, nup, k, i, false, false,
                                   Wc + WC::pt + (k * N + i) * 8, P[Ly::jee_c + k * N + i], P[Ly::jee_a + k * N + i]);
        }
        __syncthreads();
      }
      return;
    }
    jve = sm[SM::R + lane];
  }

  AQ_PH(2);
  // ------------------------------------------------------------------ F4 h-stream layers (values)
  // lane = 4i + f (electron i, unit f): h^l[i][f] stays in a register across layers; the
  // spin-group means are class sums over lanes of equal f; the four lanes of electron i
  // share its conv outputs through quad DPP sums (no LDS round trip, no barrier).
  T* hl = sm + SM::hl;
  T* cqv = sm + SM::cq;
  T* sv = sm + SM::sv;
  // fwd_reg: this lane's conv outputs (its own output of each full quad, then the Q mod 4 outputs
  // every lane evaluates) and single-layer output per layer, kept for B2
  T cqr[3][2], svr[3];
  const int fi = lane >> 2, ff = lane & 3;
  const bool ilive = fi < N;
  const int ic = ilive ? fi : N - 1;
  const bool inG1 = ic >= nup;
  T hreg = T(0);
  // fp32 proposals with 13 <= N <= 16 (4 rows per lane in F5's register layout = the 16x16 MFMA
  // accumulator layout): Phi = h^3 W + b on the matrix cores (F5 below).  Round 4, interleaved A/B
  // on one box (N2, 4096 walkers, µs per proposal launch): 224.2-225.1 -> 219.1-221.9, the
  // 16 orbital-weight VGPRs of the VALU form replaced by 4 (profiles/r04_s2_ab_mfma.txt)
#ifndef AQ_NO_PHI_MFMA
  constexpr bool phi_mfma = PROP && sizeof(T) == 4 && (N + 3) / 4 == 4 && NH == 4;
#else
  constexpr bool phi_mfma = false;
#endif
  // PROP: F5's orbital-weight column (lane column ccl of the spin-stacked [W_up; W_down] and both
  // biases), issued during F4's last layer so that F5 finds it loaded
  using V2o = typename Pair<T>::type;
  V2o ow[8], obs[2];
  T owm[4];   // phi_mfma: the MFMA B operand W_s[f = lane >> 4][c = lane & 15] (re, im) of both spins
  auto orb_load = [&]() {
    const int cl = (lane & 15) < N ? (lane & 15) : N - 1;
    const cptr<T> wcol = P + 2 * cl;
    if constexpr (phi_mfma) {
      const int fq = lane >> 4;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        owm[2 * s] = wcol[Ly::orb_w + (s * 4 + fq) * N * 2];
        owm[2 * s + 1] = wcol[Ly::orb_w + (s * 4 + fq) * N * 2 + 1];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) ow[s] = pair_make<T>(wcol[Ly::orb_w + s * N * 2], wcol[Ly::orb_w + s * N * 2 + 1]);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) obs[s] = pair_make<T>(wcol[Ly::orb_b + s * N * 2], wcol[Ly::orb_b + s * N * 2 + 1]);
  };
  if (!AQ_ABL(2)) {
#ifndef AQ_F4_NO_PRELOAD
  // this lane's layer weights (electron ic's conv weights and biases at unit ff, the single
  // layer's column ff), layer l + 1's issued before layer l's arithmetic so that their latency
  // overlaps it (left alone the compiler issues each layer's loads at their first use)
  T wcv[3][SM::QM], wcb[3][SM::QM], wsw[3][SM::QM], wsb[3];
  auto lw_load = [&](int l) {
    const int d1 = l == 0 ? D0 : NH;
    const int DF = 3 * d1 + 8;
    const int Q = DF / 4;
    const cptr<T> cw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2)) + ic * DF;
    const cptr<T> cb = P + (l == 0 ? Ly::conv_b0 : (l == 1 ? Ly::conv_b1 : Ly::conv_b2)) + ic * Q;
    const cptr<T> sw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
    const cptr<T> sb = P + (l == 0 ? Ly::sng_b0 : (l == 1 ? Ly::sng_b1 : Ly::sng_b2));
    if constexpr (xlane) {
      // the lane's records of the lane-order blocks: 2 + 2 + 1 sixteen-byte loads
      T cw8[Ly::XQ], sw8[Ly::XQ], cb4[Ly::XB];
      if (l == 0) {
        ld_use<T, Ly::XQ, Ly::Q0>(P + Ly::xcw(l) + (ic * 4 + ff) * Ly::XQ, cw8);
        ld_use<T, Ly::XQ, Ly::Q0>(P + Ly::xsw(l) + ff * Ly::XQ, sw8);
        ld_use<T, Ly::XB, Ly::CBN(Ly::Q0)>(P + Ly::xcb(l) + (ic * 4 + ff) * Ly::XB, cb4);
      } else {
        ld_use<T, Ly::XQ, Ly::Q1>(P + Ly::xcw(l) + (ic * 4 + ff) * Ly::XQ, cw8);
        ld_use<T, Ly::XQ, Ly::Q1>(P + Ly::xsw(l) + ff * Ly::XQ, sw8);
        ld_use<T, Ly::XB, Ly::CBN(Ly::Q1)>(P + Ly::xcb(l) + (ic * 4 + ff) * Ly::XB, cb4);
      }
#pragma unroll
      for (int q = 0; q < SM::QM; ++q)
        if (q < Q) {
          wcv[l][q] = cw8[q];
          wsw[l][q] = sw8[q];
        }
#pragma unroll
      for (int s4 = 0; s4 < SM::QM / 4; ++s4)
        if (s4 < Q / 4) wcb[l][s4] = cb4[s4];
#pragma unroll
      for (int q = 0; q < SM::QM; ++q)
        if (q >= 4 * (Q / 4) && q < Q) wcb[l][q] = cb4[Q / 4 + q - 4 * (Q / 4)];
    } else {
#pragma unroll
    for (int q = 0; q < SM::QM; ++q)
      if (q < Q) {
        wcv[l][q] = cw[4 * q + ff];
        wsw[l][q] = sw[q * 4 + ff];
      }
    // conv biases: lane f's output of each full quad, then the Q mod 4 outputs every lane evaluates
#pragma unroll
    for (int s4 = 0; s4 < SM::QM / 4; ++s4)
      if (s4 < Q / 4) wcb[l][s4] = cb[4 * s4 + ff];
#pragma unroll
    for (int q = 0; q < SM::QM; ++q)
      if (q >= 4 * (Q / 4) && q < Q) wcb[l][q] = cb[q];
    }
    wsb[l] = sb[ff];
  };
  lw_load(0);
#endif
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
#ifndef AQ_F4_NO_PRELOAD
    (void)convw; (void)convb; (void)sngw; (void)sngb;  // the preloaded registers replace them
    if (l + 1 < 3) lw_load(l + 1);
#ifndef AQ_F5_NO_PRELOAD
    if constexpr (PROP) {
      if (l == 2) orb_load();
    }
#endif
    asm volatile("" ::: "memory");
#define AQ_CW(q) wcv[l][q]
#define AQ_CB(s4) wcb[l][s4]
#define AQ_CR(q) wcb[l][q]
#define AQ_SW(q) wsw[l][q]
#define AQ_SB() wsb[l]
#else
#define AQ_CW(q) convw[4 * (q) + ff]
#define AQ_CB(s4) convb[4 * (s4) + ff]
#define AQ_CR(q) convb[q]
#define AQ_SW(q) sngw[(q) * 4 + ff]
#define AQ_SB() sngb[ff]
#endif
    // conv output q = tanh(mean_4(f w) + b) over the input quad 4q..4q+3
    // (network_blocks.py:106-116): lane f of electron ic holds input 4q + f (h^l unit
    // 4t + f, a group mean of unit 4t + f, or a g2 unit f) and the quad adds the four
    // products by DPP, so each product is computed once
    T hown[D0 / 4];
    if (l == 0) {
#pragma unroll
      for (int t = 0; t < D0 / 4; ++t) hown[t] = hl[ic * D0 + ff + 4 * t];
    } else {
#pragma unroll
      for (int t = 0; t < D0 / 4; ++t) hown[t] = hreg;
    }
    T gown[2][D0 / 4];
#pragma unroll
    for (int t = 0; t < D0 / 4; ++t) {
      if (t < T4) {
        const T x = ilive ? hown[t] : T(0);
        gown[0][t] = class4_sum(inG1 ? T(0) : x) * ginv0;
        gown[1][t] = class4_sum(inG1 ? x : T(0)) * ginv1;
      }
    }
    T zc[SM::QM];
#pragma unroll
    for (int q = 0; q < SM::QM; ++q) {
      if (q < Q) {
        T F;
        if (q < T4) F = hown[q];
        else if (q < 3 * T4) F = gown[(q - T4) / T4][(q - T4) % T4];
        else F = g2[((l * 2 + (q - 3 * T4)) * N + ic) * 4 + ff];
        T z = F * AQ_CW(q);
#ifndef AQ_NO_CONV_FOLD
        // opaque product: otherwise z + dpp(z) is contracted into fma(F, w, dpp(z)) and the DPP
        // move cannot fold into the add (v_mul + v_mov_dpp + v_fmac instead of v_mul + v_add_dpp)
        asm volatile("" : "+v"(z));
#endif
        z += dpp<0xB1>(z);
        z += dpp<0x4E>(z);
        zc[q] = z;
      }
    }
    // the tanh's of a full quad of outputs 4s..4s+3 are spread over the quad (lane f
    // evaluates output 4s + f, one transcendental pair instead of four) and broadcast
    // back by DPP; the Q mod 4 remaining outputs are evaluated by every lane
    const int QF = Q / 4;
    T cq[SM::QM];
#pragma unroll
    for (int s4 = 0; s4 < SM::QM / 4; ++s4) {
      if (s4 < QF) {
        const int q0 = 4 * s4;
#ifndef AQ_F4_BRANCH_SELECT
        // the four quad sums are complete before the selection: left to itself the compiler sinks
        // their last DPP add into divergent branches (exec-mask save/restore per output lane)
        T z0 = zc[q0], z1 = zc[q0 + 1], z2 = zc[q0 + 2], z3 = zc[q0 + 3];
        asm volatile("" : "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));
        const T zs = (ff & 2) ? ((ff & 1) ? z3 : z2) : ((ff & 1) ? z1 : z0);
#else
        const T zs = ff == 0 ? zc[q0] : (ff == 1 ? zc[q0 + 1] : (ff == 2 ? zc[q0 + 2] : zc[q0 + 3]));
#endif
        const T c = f_tanh(zs * T(0.25) + AQ_CB(s4));
        if constexpr (fwd_reg) cqr[l][s4] = c;
        else if (ilive) cqv[SM::cqo(l, ic) + q0 + ff] = c;
        cq[q0 + 0] = quad_bcast<0>(c);
        cq[q0 + 1] = quad_bcast<1>(c);
        cq[q0 + 2] = quad_bcast<2>(c);
        cq[q0 + 3] = quad_bcast<3>(c);
      }
    }
#pragma unroll
    for (int q = 0; q < SM::QM; ++q) {
      if (q >= 4 * QF && q < Q) {
        cq[q] = f_tanh(zc[q] * T(0.25) + AQ_CR(q));
        if constexpr (fwd_reg) cqr[l][QF + q - 4 * QF] = cq[q];
        else if (ilive && (q & 3) == ff) cqv[SM::cqo(l, ic) + q] = cq[q];
      }
    }
    T z = AQ_SB(), z1 = T(0);   // even / odd q: two independent chains
#pragma unroll
    for (int q = 0; q < SM::QM; ++q)
      if (q < Q) {
        if (q & 1) z1 += cq[q] * AQ_SW(q);
        else z += cq[q] * AQ_SW(q);
      }
    z += z1;
    const T sval = f_tanh(z);
    if constexpr (fwd_reg) svr[l] = sval;
    else if (ilive) sv[(l * N + ic) * 4 + ff] = sval;
    const T hin = l == 0 ? hl[ic * D0 + ff] : hreg;
    hreg = (d1 == NH) ? (hin + sval) * RSQ2 : sval;
#undef AQ_CW
#undef AQ_CB
#undef AQ_CR
#undef AQ_SW
#undef AQ_SB
  }
  }
  if (ilive) hl[SM::hoff(3) + ic * 4 + ff] = hreg;
  AQ_SYNC();
  if ((reuse || wfix) && lane < (wfix ? 3 * N + 2 : 2 * N + 2)) sm[SM::pv + lane] = pvr;   // read by the Gauss-Jordan after the Phi barrier
  if constexpr (PROP) {
    // F5's slot table: slot k (pivot step k) holds row r = rec[k]; it records the offsets of
    // that row's Yt row and of its h^3 row (electron rowsrc[r]) in the half of the
    // spin-stacked orbital weights that applies (the other half reads the zero row), so that
    // forming Phi needs no per-row spin selection and no row-table load
    const int r = (int)pvr;
    const int src = __shfl(rsl, lane < N ? r : 0);
    if (lane < 4 * SM::RW) {
      const bool ok = lane < N;
      const bool up = r < nup;
      const int h = SM::hl + SM::hoff(3) + src * 4;
      int* stab = (int*)(sm + SM::st) + 4 * lane;
      stab[0] = ok ? SM::yv + r * N : SM::yv;
      stab[1] = (ok && up) ? h : SM::zr;
      stab[2] = (ok && !up) ? h : SM::zr;
      stab[3] = ok ? (up ? 0 : 1) : 2;
    }
    if (lane < 4) sm[SM::zr + lane] = T(0);
    AQ_SYNC();
  }

  AQ_PH(3);
  // ------------------------------------------------------------------ F5 Phi, A = Phi * Yt, Gauss-Jordan -> B = A^{-1}
  T* Ph = sm + SM::ph;
  T* Mx = sm + SM::mx;
  const T* H3 = hl + SM::hoff(3);
  // proposals: Phi is formed in the fixed-pivot Gauss-Jordan's register layout below (no LDS
  // round trip, no barrier); the general path keeps the LDS copy for gj_inverse
  for (int idx = PROP ? N * N : lane; idx < N * N; idx += 64) {
    const int r = idx / N, col = idx - r * N;
    const int src = rowsrc[r];
    const int sp = r < nup ? 0 : 1;
    T re = T(0), im = T(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const T hv = H3[src * 4 + f];
      re += hv * P[Ly::orb_w + ((sp * 4 + f) * N + col) * 2 + 0];
      im += hv * P[Ly::orb_w + ((sp * 4 + f) * N + col) * 2 + 1];
    }
    re += P[Ly::orb_b + (sp * N + col) * 2 + 0];
    im += P[Ly::orb_b + (sp * N + col) * 2 + 1];
    Ph[idx * 2 + 0] = re;
    Ph[idx * 2 + 1] = im;
  }
  if constexpr (!PROP) AQ_SYNC();   // PROP: one wave, the Gauss-Jordan below forms Phi itself
  T logdet, phr, phi;
#ifndef AQ_NO_YBAR_REG
  constexpr bool ybar_reg = PROP;
#else
  constexpr bool ybar_reg = false;
#endif
  // PROP: the Gauss-Jordan's register block, after it X = (P A)^{-1}: lane 16 rg + c holds
  // X[4 rg + t][c] = B[4 rg + t][rec[c]] in a2[t] (gj.h), kept for B1's Yt adjoint
  V2o a2[(N + 3) / 4];
  // compact: Phi[rec[rg RW + t]][c] of lane 16 rg + c, kept for B1 / the fallback
  V2o phr4[(N + 3) / 4];
  if (reuse) {
    // the walker's pivot order (partial pivoting rerun only if a pivot comes out small)
    bool bad = false;
    logdet = phr = phi = T(0);
    if constexpr (PROP) {
      // A[r][c] = Phi[r][c] Yt[r][c] for the lane's rows r = rec[rg RW + t] (column c = lane & 15),
      // Phi[r][c] = h3[rowsrc[r]] . W_{s(r)}[:, c] + b_{s(r)}[c]; Phi also to LDS for B1
      constexpr int RW = (N + 3) / 4;
      using V2 = typename Pair<T>::type;
      const int cc = lane & 15, rg = lane >> 4;
      const T* rec = sm + SM::pv;
      const int ccl = cc < N ? cc : N - 1;
      // column ccl of the spin-stacked orbital weights [W_up; W_down] and both biases, loaded
      // once at compile-time offsets from one lane base
#if defined(AQ_F5_NO_PRELOAD) || defined(AQ_F4_NO_PRELOAD)
      orb_load();
#endif
      const V2* w = ow;
      const V2* bsp = obs;
      const int* stab = (const int*)(sm + SM::st) + 4 * RW * rg;
      if constexpr (phi_mfma) {
        // Phi[slot][c] = sum_f h3[slot][f] W_s[f][c] + b_s[c] as two K = 4 steps (one per spin) of
        // v_mfma_f32_16x16x4f32 per component: A[i = slot][k = f] = h^3 of the slot's electron
        // (the zero row for the other spin), B[k = f][j = c] = W_s[f][c], C = the slot's bias;
        // accumulator v of lane 16 rg + c is Phi[slot 4 rg + v][c], a2's layout (nn.py:432-456)
        typedef float v4f __attribute__((ext_vector_type(4)));
        const int* sti = (const int*)(sm + SM::st) + 4 * (lane & 15);
        const int fq = lane >> 4;
        const float hu = sm[sti[1] + fq], hd = sm[sti[2] + fq];
        int yo4[RW], fl4[RW];
        v4f pre, pim;
#pragma unroll
        for (int t = 0; t < RW; ++t) {
          yo4[t] = stab[4 * t];
          fl4[t] = stab[4 * t + 3];
          pre[t] = fl4[t] == 1 ? pair_re<T>(bsp[1]) : pair_re<T>(bsp[0]);
          pim[t] = fl4[t] == 1 ? pair_im<T>(bsp[1]) : pair_im<T>(bsp[0]);
        }
        pre = __builtin_amdgcn_mfma_f32_16x16x4f32(hu, owm[0], pre, 0, 0, 0);
        pim = __builtin_amdgcn_mfma_f32_16x16x4f32(hu, owm[1], pim, 0, 0, 0);
        pre = __builtin_amdgcn_mfma_f32_16x16x4f32(hd, owm[2], pre, 0, 0, 0);
        pim = __builtin_amdgcn_mfma_f32_16x16x4f32(hd, owm[3], pim, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < RW; ++t) {
          const bool ok = fl4[t] != 2 && cc < N;
          if constexpr (compact) {
            phr4[t] = pair_make<T>(pre[t], pim[t]);
          } else if (ok) {
            const int e = yo4[t] - SM::yv + cc;   // r N + c
            Ph[e * 2 + 0] = pre[t];
            Ph[e * 2 + 1] = pim[t];
          }
          const T y = ok ? sm[yo4[t] + ccl] : T(0);
          a2[t] = pair_make<T>(pre[t] * y, pim[t] * y);
        }
      } else
#pragma unroll
      for (int t = 0; t < RW; ++t) {
        const int yo = stab[4 * t], hu = stab[4 * t + 1], hd = stab[4 * t + 2], fl = stab[4 * t + 3];
        V2 acc = fl == 1 ? bsp[1] : bsp[0];
#pragma unroll
        for (int f = 0; f < 4; ++f) acc = pair_fma<T>(sm[hu + f], w[f], acc);
#pragma unroll
        for (int f = 0; f < 4; ++f) acc = pair_fma<T>(sm[hd + f], w[4 + f], acc);
        const bool ok = fl != 2 && cc < N;
        if constexpr (compact) {
          phr4[t] = acc;
        } else if (ok) {
          const int e = yo - SM::yv + cc;   // r N + c
          Ph[e * 2 + 0] = pair_re<T>(acc);
          Ph[e * 2 + 1] = pair_im<T>(acc);
        }
        const T y = ok ? sm[yo + ccl] : T(0);
        a2[t] = pair_make<T>(pair_re<T>(acc) * y, pair_im<T>(acc) * y);
      }
      // the elimination and B2 (below) run at raised wave priority: dense VALU with short
      // dependencies, issued ahead of co-resident waves in their load/LDS-bound phases
      // (measured: 224.7-226.3 -> 221.1-221.6 us per N2 launch; F4 too, B3, or the F1 load issue
      // were neutral or worse)
#ifndef AQ_NO_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
      if (!AQ_ABL(4)) gj_fixed_regs<T, N>(a2, Mx, lane, rec, logdet, phr, phi, bad);
#ifndef AQ_NO_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    } else
    if (!AQ_ABL(4)) gj_inverse_fixed<T, N>(Ph, Yv, Mx, lane, sm + SM::pv, logdet, phr, phi, bad);
#ifdef AQ_ABLATE
    if (ka.ablate) bad = false;
#endif
    if (bad) {
#ifdef AQ_PHASE_PROF
      if (lane == 0) atomicAdd(&aq_phase_cycles[15], 1ull);   // fallback count (diagnostics build)
#endif
#ifdef AQ_PHASE_MARK
      AQ_PH(10);   // tools/isa_phases.py: the rarely taken pivoted fallback, counted apart
#endif
      if constexpr (compact) {
        // compact layout: no Phi block in LDS; the pivoted inverse reads Phi from the B block it
        // then overwrites (gj_inverse loads its whole input before it writes)
        wave_sync();
        const int cc = lane & 15, rg = lane >> 4;
        constexpr int RW = (N + 3) / 4;
#pragma unroll
        for (int t = 0; t < RW; ++t) {
          const int i = rg * RW + t;
          if (i < N && cc < N) {
            const int r = (int)sm[SM::pv + i];
            Mx[(r * N + cc) * 2] = pair_re<T>(phr4[t]);
            Mx[(r * N + cc) * 2 + 1] = pair_im<T>(phr4[t]);
          }
        }
        wave_sync();
        gj_inverse<T, N>(Mx, Yv, Mx, lane, logdet, phr, phi);
      } else {
        gj_inverse<T, N>(Ph, Yv, Mx, lane, logdet, phr, phi);
      }
      if constexpr (ybar_reg && !compact) {
        // the register block of B for B1, from the pivoted inverse (natural layout in Mx)
        wave_sync();
        const int cc = lane & 15, rg = lane >> 4;
        const int r = (int)sm[SM::pv + (cc < N ? cc : 0)];
#pragma unroll
        for (int t = 0; t < (N + 3) / 4; ++t) {
          const int c = rg * ((N + 3) / 4) + t;
          const int e = ((c < N ? c : 0) * N + r) * 2;
          a2[t] = pair_make<T>(Mx[e], Mx[e + 1]);
        }
      }
#ifdef AQ_PHASE_MARK
      AQ_PH(11);
#endif
    }
  } else {
    // walker launches after an mc_step's first sweep: the previous sweep's pivot order (no pivot
    // search: gj_inverse's per-step argmax over the column is most of its latency), log|det| from
    // this matrix's own pivots, the record's magnitudes refreshed for the proposals; the pivoted
    // elimination if a pivot comes out below 0.1 of the previous one (it then rewrites the record)
    bool bad = true;
    if (wfix) gj_inverse_fixed<T, N>(Ph, Yv, Mx, lane, sm + SM::pv, logdet, phr, phi, bad, Wc + WC::pv, 2 * N + 2);
    if (bad) gj_inverse<T, N>(Ph, Yv, Mx, lane, logdet, phr, phi, (!PREP && !isprop) ? Wc + WC::pv : nullptr);
  }
  if constexpr (!PREP) {
    if (ka.value_only) {   // ECP quadrature configurations: log|psi| and phase only
      const T jsum = fwd_reg ? jsum_p : wave_sum(jv + jve);
      const T lpsi = logdet + jsum;
      if (lane == 0) {
        if (ka.logabs) ((T*)ka.logabs)[conf] = lpsi;
        if (ka.phase) ((T*)ka.phase)[conf] = f_atan2(phi, phr);
      }
      if (ka.orb) {
        // make_orbitals.apply's output (nn.py:485-506): Phi (rows = up electrons then down
        // electrons) * Yt (row r: electron r's envelope and y row, Q1) * exp(J_ee/N) exp(J_ae/N)
        const T je = wave_sum(jve), ja = wave_sum(jv);
        const T sc = f_exp(je / T(N)) * f_exp(ja / T(N));
        T* O = (T*)ka.orb + (size_t)conf * N * N * 2;
        for (int idx = lane; idx < N * N; idx += 64) {
          const T y = Yv[idx] * sc;
          O[2 * idx] = Ph[2 * idx] * y;
          O[2 * idx + 1] = Ph[2 * idx + 1] * y;
        }
      }
      return;
    }
  }
  AQ_SYNC();
#define BRE(c, s) Mx[((c) * N + (s)) * 2]
#define BIM(c, s) Mx[((c) * N + (s)) * 2 + 1]

  AQ_PH(4);
  // ------------------------------------------------------------------ B1 adjoints of H (= h^3) and Yt
  T* hbar = sm + SM::hbar;
  T* ybar = sm + SM::ybar;
#ifndef AQ_PREP_NO_MFMA
  // fp32 adjoint pass of the local energy: Q_f on the matrix cores (below), B1 from its diagonal
  constexpr bool q_mfma = PREP && sizeof(T) == 4 && NH == 4;
#else
  constexpr bool q_mfma = false;
#endif
#ifdef AQ_B1_MFMA
  // fp32 value + gradient (proposals and walker launches): B1's H adjoint on the matrix cores.
  // Opt-in, measured slower (round 4, interleaved A/B on one box, N2 4096 walkers, µs per
  // proposal launch: 230.2-233.7 with it against 219.1-221.9 without; the walker launch 50.0-50.3
  // against 49.3-49.4; profiles/r04_s2_ab_mfma.txt): the proposal instantiation spills at the
  // 5-wave budget (96 VGPRs + 16 B) and the eight dependent MFMAs serialise on one accumulator
  constexpr bool b1_mfma = !PREP && sizeof(T) == 4 && NH == 4;
#else
  constexpr bool b1_mfma = false;
#endif
  if constexpr (b1_mfma) {
    // dL/dH[r][f] = Re Q_f[r,r] = Re sum_c W_{s(r)}[f][c] G[c][r], G[c][r] = Yt[r][c] B[c][r]:
    // the (8 x N)(N x N) product [W_up; W_down] G on v_mfma_f32_16x16x4f32 (Re = W_re G_re -
    // W_im G_im, two MFMAs per K-step of four columns c = 4 k + t, k = lane >> 4); A[i = f + 4 s][k]
    // = W_s[f][c] (rows 8..15 zero), B[k][j = r] = G[c][r] from B (LDS) and Yt; accumulator v of
    // lane 16 s + r is row f = v of spin block s, kept for the rows r of spin s (nn.py:432-456)
    if (!AQ_ABL(8)) {
      typedef float v4f __attribute__((ext_vector_type(4)));
      const int j = lane & 15, kq = lane >> 4;
      const bool jok = j < N;
      const int jr = jok ? j : N - 1;
      const int si = (j >> 2) & 1, fi = j & 3;   // A row j = f + 4 s
      const bool iok = j < 8;
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = 4 * kq + t;
        const bool cok = c < N;
        const int cl = cok ? c : N - 1;
        const float wr = P[Ly::orb_w + ((si * 4 + fi) * N + cl) * 2];
        const float wi = P[Ly::orb_w + ((si * 4 + fi) * N + cl) * 2 + 1];
        const float ar = (iok && cok) ? wr : 0.f, ai = (iok && cok) ? -wi : 0.f;
        const float y = Yv[jr * N + cl];
        const bool gok = cok && jok;
        const float gr = gok ? y * (float)Mx[(cl * N + jr) * 2] : 0.f;
        const float gi = gok ? y * (float)Mx[(cl * N + jr) * 2 + 1] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar, gr, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ai, gi, acc, 0, 0, 0);
      }
      if (jok && kq == (j >= nup ? 1 : 0)) {
        const int h = SM::hoff(3) + rowsrc[j] * 4;
#pragma unroll
        for (int v = 0; v < 4; ++v) hbar[h + v] = acc[v];
      }
    }
  } else
  if (!q_mfma && lane < 4 * N && !AQ_ABL(8)) {
    const int r = lane >> 2, f = lane & 3;
    const int sp = r < nup ? 0 : 1;
    T q = T(0), q1 = T(0);   // even / odd c: two independent chains
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const T yv = Yv[r * N + c];
      const T wr = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2] * yv;
      const T wi = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1] * yv;
      // Re Q_f[r,r] (PH: Im Q_f[r,r])
      const T qc = PH ? wr * BIM(c, r) + wi * BRE(c, r) : wr * BRE(c, r) - wi * BIM(c, r);
      if (c & 1) q1 += qc;
      else q += qc;
    }
    q += q1;
    hbar[SM::hoff(3) + rowsrc[r] * 4 + f] = q;
  }
  if constexpr (PREP) {
    // B, Phi and Q_f[r,s] = sum_c W_{s(r)}[f,c] Yt[r,c] B[c,s] for the determinant terms
    for (int idx = lane; idx < 2 * N * N; idx += 64) {
      Lw[LCc::bm + idx] = Mx[idx];
      Lw[LCc::ph + idx] = Ph[idx];
    }
    if constexpr (q_mfma) {
      // Q_f = U B, U[(r, f), c] = W_{s(r)}[f, c] Yt[r, c]: a (4N x N)(N x N) complex product on
      // v_mfma_f32_16x16x4f32 (nn.py:449-485's orbital matmul): M-tiles over the rows (r, f),
      // K-steps of four columns c, one N-tile s.  A fragment: lane (k = lane >> 4, row e =
      // lane & 15); B fragment: lane (k, column e); accumulator v of lane group k: row 4k + v.
      // Replaces a VALU loop of N^3 complex MACs with two global weight loads and an LDS read
      // of Yt per MAC.  B1's H adjoint is Re Q_f[r, r] (the diagonal), written from here.
      typedef float v4f __attribute__((ext_vector_type(4)));
      constexpr int NM = (4 * N + 15) / 16, NK = (N + 3) / 4;
      const int kq = lane >> 4, e = lane & 15, fq = lane & 3;
      float bre[NK], bim[NK], wr[2][NK], wi[2][NK];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int c = 4 * kk + kq;
        const bool bok = c < N && e < N;
        const int cl = c < N ? c : N - 1, el = e < N ? e : N - 1;
        bre[kk] = bok ? (float)BRE(cl, el) : 0.f;
        bim[kk] = bok ? (float)BIM(cl, el) : 0.f;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const float a = P[Ly::orb_w + ((sp * 4 + fq) * N + cl) * 2], b = P[Ly::orb_w + ((sp * 4 + fq) * N + cl) * 2 + 1];
          wr[sp][kk] = c < N ? a : 0.f;
          wi[sp][kk] = c < N ? b : 0.f;
        }
      }
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int r = 4 * m + (e >> 2);            // A row 16 m + e = (r, f = e & 3)
        const bool rok = r < N;
        const bool up = r < nup;
        v4f qre = {0.f, 0.f, 0.f, 0.f}, qim = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int c = 4 * kk + kq;
          const float y = (rok && c < N) ? (float)Yv[(rok ? r : 0) * N + (c < N ? c : 0)] : 0.f;
          const float ur = (up ? wr[0][kk] : wr[1][kk]) * y, ui = (up ? wi[0][kk] : wi[1][kk]) * y;
          qre = __builtin_amdgcn_mfma_f32_16x16x4f32(ur, bre[kk], qre, 0, 0, 0);
          qre = __builtin_amdgcn_mfma_f32_16x16x4f32(-ui, bim[kk], qre, 0, 0, 0);
          qim = __builtin_amdgcn_mfma_f32_16x16x4f32(ur, bim[kk], qim, 0, 0, 0);
          qim = __builtin_amdgcn_mfma_f32_16x16x4f32(ui, bre[kk], qim, 0, 0, 0);
        }
        const int rr = 4 * m + kq;                 // accumulator rows 4 kq + v: (rr, f = v), column s = e
        if (rr < N && e < N) {
          T* dst = Lw + LCc::qs + (rr * N + e) * 8;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            dst[2 * v] = qre[v];
            dst[2 * v + 1] = qim[v];
          }
          if (e == rr && !AQ_ABL(8)) {
#pragma unroll
            for (int v = 0; v < 4; ++v) hbar[SM::hoff(3) + rowsrc[rr] * 4 + v] = PH ? qim[v] : qre[v];
          }
        }
      }
    } else {
    for (int idx = lane; idx < NH * N * N; idx += 64) {
      const int rs = idx >> 2, f = idx & 3;
      const int r = rs / N, s = rs - r * N;
      const int sp = r < nup ? 0 : 1;
      T qr = T(0), qi = T(0);
      for (int c = 0; c < N; ++c) {
        const T yv = Yv[r * N + c];
        const T wr = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2] * yv;
        const T wi = P[Ly::orb_w + ((sp * 4 + f) * N + c) * 2 + 1] * yv;
        qr += wr * BRE(c, s) - wi * BIM(c, s);
        qi += wr * BIM(c, s) + wi * BRE(c, s);
      }
      Lw[LCc::qs + idx * 2] = qr;
      Lw[LCc::qs + idx * 2 + 1] = qi;
    }
    }
  }
  AQ_SYNC();   // ybar overwrites Yt
  if constexpr (compact) {
    // dL/dYt[r][c] = Re(B[c][r] Phi[r][c]) with Phi from F5's registers (lane 16 rg + c, slot
    // rg RW + t, r = rec[slot]) and B from LDS
    if (!AQ_ABL(8)) {
      const int cc = lane & 15, rg = lane >> 4;
      constexpr int RW = (N + 3) / 4;
      if (cc < N) {
#pragma unroll
        for (int t = 0; t < RW; ++t) {
          const int i = rg * RW + t;
          if (i < N) {
            const int r = (int)sm[SM::pv + i];
            const int e = r * N + cc;
            ybar[e] = Mx[(cc * N + r) * 2] * pair_re<T>(phr4[t]) - Mx[(cc * N + r) * 2 + 1] * pair_im<T>(phr4[t]);
          }
        }
      }
    }
  } else
  if constexpr (ybar_reg) {
    // dL/dYt[r][c] = Re(B[c][r] Phi[r][c]) from the register block: B[c][r] = a2[t] of lane
    // 16 rg + cc with c = 4 rg + t, r = rec[cc] (no B reads, no per-element index division)
    if (!AQ_ABL(8)) {
      const int cc = lane & 15, rg = lane >> 4;
      constexpr int RW = (N + 3) / 4;
      if (cc < N) {
        const int r = (int)sm[SM::pv + cc];
#pragma unroll
        for (int t = 0; t < RW; ++t) {
          const int c = rg * RW + t;
          if (c < N) {
            const int e = r * N + c;
            ybar[e] = pair_re<T>(a2[t]) * Ph[e * 2] - pair_im<T>(a2[t]) * Ph[e * 2 + 1];
          }
        }
      }
    }
  } else
  if constexpr (!PREP) {
    if (!AQ_ABL(8)) {
      for (int idx = lane; idx < N * N; idx += 64) {
        const int r = idx / N, c = idx - r * N;
        ybar[idx] = BRE(c, r) * Ph[idx * 2] - BIM(c, r) * Ph[idx * 2 + 1];
      }
    }
  }
#undef BRE
#undef BIM
  AQ_SYNC();

  AQ_PH(5);
  // ------------------------------------------------------------------ B2 back through the h-stream layers
  // lane map of F4: the adjoint of h^{l+1}[i][f] stays in a register.
  T* g2b = sm + SM::g2;    // forward g2 values are dead after F4: reuse for their adjoints
#ifndef AQ_NO_PRIO
  if constexpr (PROP) __builtin_amdgcn_s_setprio(1);
#endif
  if (!AQ_ABL(16)) {
#ifdef AQ_B2_PRELOAD
    // as in F4: this lane's layer weights (the single layer's rows of the conv outputs this lane
    // forms, electron ic's conv weights at unit ff), layer l - 1's issued before layer l
    T bsw[3][SM::QM / 4][4], bcw[3][SM::QM];
    auto bw_load = [&](int l) {
      const int d1 = l == 0 ? D0 : NH;
      const int DF = 3 * d1 + 8;
      const int Q = DF / 4;
      const cptr<T> cw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2)) + ic * DF;
      const cptr<T> sw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
#pragma unroll
      for (int s4 = 0; s4 < SM::QM / 4; ++s4)
        if (s4 < Q / 4)
#pragma unroll
          for (int m = 0; m < 4; ++m) bsw[l][s4][m] = sw[(4 * s4 + ff) * 4 + m];
#pragma unroll
      for (int q = 0; q < SM::QM; ++q)
        if (q < Q) bcw[l][q] = cw[4 * q + ff];
    };
    bw_load(2);
#endif
    T hb = hbar[SM::hoff(3) + ic * 4 + ff];
#pragma unroll
    for (int l = 2; l >= 0; --l) {
      const int d1 = l == 0 ? D0 : NH;
      const int DF = 3 * d1 + 8;
      const int Q = DF / 4;
      const int T4 = d1 / 4;
      const cptr<T> convw = P + (l == 0 ? Ly::conv_w0 : (l == 1 ? Ly::conv_w1 : Ly::conv_w2)) + ic * DF;
      const cptr<T> sngw = P + (l == 0 ? Ly::sng_w0 : (l == 1 ? Ly::sng_w1 : Ly::sng_w2));
#ifdef AQ_B2_PRELOAD
      if (l > 0) bw_load(l - 1);
      asm volatile("" ::: "memory");
#endif
      // single: s = tanh(c Ws + b), h_out = res(h_in, s)
      const T sval = fwd_reg ? svr[l] : sv[(l * N + ic) * 4 + ff];
      const T sb = (d1 == NH) ? hb * RSQ2 : hb;
      const T zs = sb * (T(1) - sval * sval);
      if constexpr (PREP) {
        // single node: tanh' and the curvature weight abar * tanh''(z) = sb * (-2 s (1 - s^2))
        if (ilive) {
          T* sn = Lw + l * LCc::layer_n + LCc::sn + (ic * NH + ff) * 2;
          sn[0] = T(1) - sval * sval;
          sn[1] = T(-2) * sval * zs;
        }
      }
      const T zq[4] = {quad_bcast<0>(zs), quad_bcast<1>(zs), quad_bcast<2>(zs), quad_bcast<3>(zs)};
      // conv: c = tanh(0.25 sum F w + b); fb[q] = adjoint of input 4q + f
      // cg[q] = tanh'(conv q) * 0.25 * (adjoint of conv output q) is the same on the four
      // lanes of an electron: for a full quad of outputs 4s..4s+3 lane f forms output 4s + f
      // and DPP broadcasts it (as the forward tanh's); the Q mod 4 rest on every lane
      const int QF = Q / 4;
      T cg[SM::QM];
      T bcw8[Ly::XQ];   // kXLane: this lane's conv weights (electron ic, unit ff), 2 sixteen-byte loads
      if constexpr (xlane) {
        if (l == 0) ld_use<T, Ly::XQ, Ly::Q0>(P + Ly::xcw(l) + (ic * 4 + ff) * Ly::XQ, bcw8);
        else ld_use<T, Ly::XQ, Ly::Q1>(P + Ly::xcw(l) + (ic * 4 + ff) * Ly::XQ, bcw8);
      }
#pragma unroll
      for (int q = 0; q < SM::QM; ++q) {
        const bool full = q < 4 * QF;
        if (q < Q && (!full || (q & 3) == 0)) {
          const int qq = full ? q + ff : q;     // output this lane forms
          T cb = T(0);
          T srow[4];   // kXLane: single-layer weight row qq, one sixteen-byte load
          if constexpr (xlane) ld_vec<T, 4>(P + Ly::xsr(l) + qq * 4, srow);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
#ifdef AQ_B2_PRELOAD
            cb += zq[m] * (full ? bsw[l][q / 4][m] : sngw[qq * 4 + m]);
#else
            cb += zq[m] * (xlane ? srow[m] : sngw[qq * 4 + m]);
#endif
          }
          const T c = fwd_reg ? cqr[l][full ? q / 4 : QF + q - 4 * QF] : cqv[SM::cqo(l, ic) + qq];
          const T g = cb * (T(1) - c * c) * T(0.25);
          if constexpr (PREP) {
            // conv node (stored once, by the lane of its quad position): tanh', abar * tanh''
            // (pre-scaled by the conv's 1/4 and its square: k_walker_lap multiplies the unscaled sum,
            // the same products bit for bit since the scalings are powers of two)
            if (ilive && (qq & 3) == ff) {
              const T c1 = T(1) - c * c;
              T* cn = Lw + l * LCc::layer_n + LCc::cn + (ic * LCc::QM + qq) * 2;
              cn[0] = c1 * T(0.25);
              cn[1] = (T(-2) * c * c1 * cb) * T(0.0625);
            }
          }
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
      T fb[SM::QM];
#pragma unroll
      for (int q = 0; q < SM::QM; ++q)
#ifdef AQ_B2_PRELOAD
        if (q < Q) fb[q] = cg[q] * bcw[l][q];
#else
        if (q < Q) fb[q] = cg[q] * (xlane ? bcw8[q] : convw[4 * q + ff]);
#endif
      // g2 adjoints (inputs 3 d1 + 4G + f), consumed by B3
      if (ilive) {   // pre-scaled by the group-mean weights 1/|G| of the pair sums
        g2b[((l * 2 + 0) * N + ic) * 4 + ff] = fb[3 * T4 + 0] * ginv0;
        g2b[((l * 2 + 1) * N + ic) * 4 + ff] = fb[3 * T4 + 1] * ginv1;
      }
      // group-mean adjoints and h^l adjoints of units m = f + 4t
      T hn = T(0);
#pragma unroll
      for (int t = 0; t < D0 / 4; ++t) {
        if (t < T4) {
          const T s0 = class4_sum(ilive ? fb[T4 + t] : T(0)) * ginv0;
          const T s1 = class4_sum(ilive ? fb[2 * T4 + t] : T(0)) * ginv1;
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
  AQ_SYNC();
#ifndef AQ_NO_PRIO
  if constexpr (PROP) __builtin_amdgcn_s_setprio(0);
#endif

  if constexpr (PREP) {
    // ---------------------------------------------------------------- local-energy adjoint pass: tail
    for (int idx = lane; idx < N * D0; idx += 64) Lw[LCc::h0b + idx] = hbar[idx];
    // Pair stream, lane 4 i + kq: column i, the pairs (k, i) with k = kq mod 4 of one spin group at
    // a time; each pair's forward values through the double layers once, with the first and second
    // derivatives along the three components d_c of d = x_i - x_k carried together.
    //  * sd[l][G][i][c][f] = sum_{k in G, k != i} d h2^{(l)}[k,i][f] / d d_c  (k_walker_lap: the
    //    derivative of the column mean g2 along x_{i,c}), summed over the four lanes of column i;
    //  * pair-local Laplacian: sum over the pair terms of g2 of their adjoint (g2b, already
    //    scaled by 1/|G|) times their Laplacian in (x_k, x_i) = 2 sum_c d^2/d d_c^2.
    // Round 4: the (direction, column) lane layout ran the 14 pairs of a column serially on each
    // direction lane and recomputed the forward values per direction (≈ 3,000 of the launch's
    // 7,765 VALU instructions per wave).
    const int ci = lane >> 2, kq = lane & 3;
    const bool ilv = ci < N;
    const int ii = ilv ? ci : N - 1;
    T pcurv = T(0);
    // directions C0 .. C0 + NC - 1 together (two passes, {0, 1} and {2}: the three together spill
    // at the 4-waves/SIMD register budget)
    auto pair_pass = [&](auto c0_, auto nc_) {
      constexpr int C0 = decltype(c0_)::value, NC = decltype(nc_)::value;
#pragma unroll 1
      for (int G = 0; G < 2; ++G) {
        const int k0 = G ? nup : 0, k1 = G ? N : nup;
        const T* gb = g2b + (G * N + ii) * 4;        // level l at + l * 2 * N * 4
        T s0[NC];           // level 0: sum of u_c = d_c / r (the other three features count the pairs)
        T s1[2][NC][4];     // levels 1, 2
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          s0[c] = T(0);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int f = 0; f < 4; ++f) s1[j][c][f] = T(0);
        }
        // the pair's double-layer tanh's: written by this lane in F2 (LapCache pt, same (k, i) per lane),
        // read back one pair ahead instead of re-running the value chain in each pass
        const int kfirst = k0 + ((kq - k0) & 3);
        const T* tpb = Lw + LCc::pt + ii * LCc::pt_n;
        T tq[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) tq[o] = tpb[(kfirst < k1 ? kfirst : k0) * N * LCc::pt_n + o];
#pragma unroll 1
        for (int k = kfirst; k < k1; k += 4) {
          const bool dg = (k == ii);
          const T m = (ilv && !dg) ? T(1) : T(0);
          T tcur[8];
#pragma unroll
          for (int o = 0; o < 8; ++o) tcur[o] = tq[o];
#pragma unroll
          for (int o = 0; o < 8; ++o) tq[o] = tpb[(k + 4 < k1 ? k + 4 : k) * N * LCc::pt_n + o];
          T d[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) d[c] = xs[ii * 3 + c] - xs[k * 3 + c];
          const T r = f_sqrt(dg ? T(1) : d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
          const T ir = f_rcp(r);
          T p1[NC][4], p2[NC][4];
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const T u = d[C0 + c] * ir;
            p1[c][0] = u;
#pragma unroll
            for (int f = 1; f < 4; ++f) p1[c][f] = (f - 1 == C0 + c) ? T(1) : T(0);
            p2[c][0] = (T(1) - u * u) * ir;
#pragma unroll
            for (int f = 1; f < 4; ++f) p2[c][f] = T(0);
            s0[c] += m * u;
            pcurv += m * gb[0] * p2[c][0];             // level 0: only r has curvature
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const cptr<T> dw = P + (j == 0 ? Ly::dbl_w0 : Ly::dbl_w1);
            const T* gl = gb + (j + 1) * 2 * N * 4;
            T tv[4];
#pragma unroll
            for (int o = 0; o < 4; ++o) tv[o] = tcur[j * 4 + o];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              T z1[4], z2[4];
#pragma unroll
              for (int o = 0; o < 4; ++o) {
                T a1 = T(0), a2 = (j == 0) ? p2[c][0] * dw[o] : T(0);
#pragma unroll
                for (int mm = 0; mm < 4; ++mm) {
                  a1 += p1[c][mm] * dw[mm * 4 + o];
                  if (j > 0) a2 += p2[c][mm] * dw[mm * 4 + o];
                }
                z1[o] = a1;
                z2[o] = a2;
              }
#pragma unroll
              for (int o = 0; o < 4; ++o) {
                const T sd1 = T(1) - tv[o] * tv[o];
                const T t1 = sd1 * z1[o];
                const T t2 = sd1 * (z2[o] - T(2) * tv[o] * z1[o] * z1[o]);
                p1[c][o] = (p1[c][o] + t1) * RSQ2;
                p2[c][o] = (p2[c][o] + t2) * RSQ2;
                s1[j][c][o] += m * p1[c][o];
                pcurv += m * gl[o] * p2[c][o];
              }
            }
          }
        }
        // column i's totals over its four lanes; lane kq stores direction C0 + kq (kq < NC)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          s0[c] += dpp<0xB1>(s0[c]);
          s0[c] += dpp<0x4E>(s0[c]);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int f = 0; f < 4; ++f) {
              s1[j][c][f] += dpp<0xB1>(s1[j][c][f]);
              s1[j][c][f] += dpp<0x4E>(s1[j][c][f]);
            }
        }
        if (ilv && kq < NC) {
          const int c = C0 + kq;
          const T cnt = T(k1 - k0 - ((ii >= k0 && ii < k1) ? 1 : 0));   // pairs (k, i), k in G, k != i
          T* o0 = Lw + LCc::sd + ((G * N + ii) * 3 + c) * 4;
          o0[0] = (NC == 1 || kq == 0) ? s0[0] : s0[NC - 1];
#pragma unroll
          for (int f = 1; f < 4; ++f) o0[f] = (f - 1 == c) ? cnt : T(0);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            T* oj = Lw + (j + 1) * LCc::layer_n + LCc::sd + ((G * N + ii) * 3 + c) * 4;
#pragma unroll
            for (int f = 0; f < 4; ++f) oj[f] = (NC == 1 || kq == 0) ? s1[j][0][f] : s1[j][NC - 1][f];
          }
        }
      }
    };
    pair_pass(std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{});
    pair_pass(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
    // x2: the second derivatives along x_{k,c} equal those along x_{i,c}
    pcurv = T(2) * wave_sum(pcurv);
    const T lpsi = logdet + wave_sum(jv + jve);
    if (lane == 0) {
      Lw[LCc::scal] = pcurv;
      if (ka.logabs) ((T*)ka.logabs)[conf] = lpsi;
      if (ka.phase) ((T*)ka.phase)[conf] = f_atan2(phi, phr);
    }
    return;
  }

  // electron-local Jacobians of this lane's (electron, direction) for B4, fetched ahead of B3:
  // from the walker cache, or the moved electron's entry of this proposal
  const int c4 = lc < 3 ? lc : 0;
  T lv[N + D0];
  auto lv_load = [&]() {
    const bool mov = reuse && le == pi;
    const T* la = mov ? Eq + EC::yd + c4 * N : Wc + WC::loc + (lane < 48 ? lane : 47);
    const T* lb = mov ? Eq + EC::hd + c4 * D0 : Wc + WC::loc + N * 48 + (lane < 48 ? lane : 47);
    const int st = mov ? 1 : 48;
#pragma unroll
    for (int m = 0; m < N; ++m) lv[m] = la[m * st];
#pragma unroll
    for (int m = 0; m < D0; ++m) lv[N + m] = lb[m * st];
  };
  // where the proposal path issues B4's Jacobian loads: 0 = before B3 (their latency overlaps all
  // of B3), k = after B3's iteration k - 1.  Round 4: 1..3 leave the fp32 N2 proposal kernel at 95
  // VGPRs and do not remove the spills of a 6-wave build (15-16 VGPRs): not the pressure point
#ifndef AQ_LV_AT
#define AQ_LV_AT 0
#endif
  constexpr int lv_at = (reuse && PROP) ? AQ_LV_AT : 0;
  if (lv_at == 0) lv_load();
  AQ_PH(6);
  // ------------------------------------------------------------------ B3 pair adjoints d(logpsi)/d(x_i - x_k)
  T* dbar = sm + SM::dbar;
  // Proposals from the walker cache: the 2(N-1) pairs of the moved electron pi come first
  // (iteration 0) and recompute their forward values; every other pair takes t1, t2
  // from walker pb's cache, so iterations >= 1 skip the forward recompute.
  // one ordered pair (k, i): forward values (fresh) or the cached t1, t2 of walker pb, then the
  // adjoints back through the two double layers to d = x_i - x_k
  auto pair_adjoint = [&](int k, int i, bool may_fresh, bool fresh, const T* tcache, T cusp, T al) {
    b3_pair_adjoint<T, N, A>(P, xs, g2b, dbar, nup, k, i, may_fresh, fresh, tcache, cusp, al);
  };
  constexpr int NPR = N * (N - 1);
  if (reuse && !AQ_ABL(32)) {
    // Proposals: iteration u of lane l is pair index it = l + 64 u.  The 2(N-1) pairs of the
    // moved electron pi (it < M, all in iteration 0) recompute their forward values; every
    // other pair takes t1, t2 from walker pb's cache.  All cached loads of the lane are issued
    // before the first pair is processed, so their latency overlaps the fresh pairs' tanh's
    // and the earlier iterations (instead of one exposed cache round trip per iteration).
    constexpr int M = 2 * (N - 1);
    constexpr int NIT = (NPR + 63) / 64;
    T tc[NIT][8], jc[NIT], ja[NIT];
    int pk[NIT], pi2[NIT];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      // pair (k, i) of this slot from the constant table (PairTab)
      const unsigned code = pair_tab<N>.v[pi][lane + 64 * u];
      const int k = code & 15, i = (code >> 4) & 15;
      pk[u] = k;
      pi2[u] = i;
      jc[u] = P[Ly::jee_c + k * N + i];
      ja[u] = P[Ly::jee_a + k * N + i];
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int k = pk[u], i = pi2[u];
      // loaded on every lane (the fresh pairs of iteration 0 select their own values)
      const T* tp = Wc + WC::pt + (k * N + i) * 8;
#pragma unroll
      for (int o = 0; o < 8; ++o) tc[u][o] = tp[o];
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int it = lane + 64 * u;
      if (it < NPR) pair_adjoint(pk[u], pi2[u], u == 0, u == 0 && it < M, tc[u], jc[u], ja[u]);
      if (lv_at == u + 1) lv_load();
    }
  } else if (!reuse) {
    if (!PREP && !isprop && ka.wcache) {
      // walker launch of a sweep: F2 has just written every pair's tanh outputs to the walker
      // cache; read them back instead of recomputing the two double layers.  SPL: wave 1 (waiting
      // at this barrier since F2) takes the odd 64-pair blocks
      if constexpr (SPL) __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      for (int it = lane; it < NPR; it += SPL ? 128 : 64) {
        const int k = it / (N - 1);
        const int jj = it - k * (N - 1);
        const int i = jj + (jj >= k ? 1 : 0);
        pair_adjoint(k, i, false, false, Wc + WC::pt + (k * N + i) * 8, P[Ly::jee_c + k * N + i], P[Ly::jee_a + k * N + i]);
      }
      if constexpr (SPL) __syncthreads();   // wave 1's share of dbar is in LDS
    } else {
      for (int it = lane; it < NPR; it += 64) {
        const int k = it / (N - 1);
        const int jj = it - k * (N - 1);
        const int i = jj + (jj >= k ? 1 : 0);
        pair_adjoint(k, i, true, true, nullptr, P[Ly::jee_c + k * N + i], P[Ly::jee_a + k * N + i]);
      }
    }
  }
  AQ_SYNC();

  AQ_PH(7);
  // ------------------------------------------------------------------ B4 gradient per direction lane (c, e)
  T g = fwd_reg ? sm[SM::jdo + lane] : jd1;
  if (!AQ_ABL(64)) {
    // four partial sums: the LDS reads and FMAs of one chain do not wait on each other
    T ga = T(0), gb = T(0), gc = T(0);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const T dk = dbar[(k * N + le) * 3 + c4] - dbar[(le * N + k) * 3 + c4];
      if (k & 1) ga += (k == le) ? T(0) : dk;
      else g += (k == le) ? T(0) : dk;
    }
#pragma unroll
    for (int col = 0; col < N; ++col) {
      if (col & 1) gc = f_fma(ybar[le * N + col], lv[col], gc);
      else gb = f_fma(ybar[le * N + col], lv[col], gb);
    }
#pragma unroll
    for (int m = 0; m < D0; ++m) {
      if (m & 1) gc = f_fma(hbar[le * D0 + m], lv[N + m], gc);
      else gb = f_fma(hbar[le * D0 + m], lv[N + m], gb);
    }
    g = (g + ga) + (gb + gc);
  }

  AQ_PH(8);
  // ------------------------------------------------------------------ outputs
  const T gd = dir ? g : T(0);
  const T sumsq = wave_sum(gd * gd);
  const T lpsi = logdet + (fwd_reg ? jsum_p : wave_sum(jv + jve));
  const auto* kl = late_args();
  if (kl->grad && dir) ((T*)kl->grad)[(size_t)conf * 3 * N + 3 * le + lc] = g;
  if (kl->gown && dir && le == pi) ((T*)kl->gown)[(size_t)conf * 3 + lc] = g;
  if (lane == 0) {
    if (kl->logabs) ((T*)kl->logabs)[conf] = lpsi;
    if (kl->phase) ((T*)kl->phase)[conf] = f_atan2(phi, phr);
    if (kl->sumsq) ((T*)kl->sumsq)[conf] = sumsq;
    if (kl->tacc) tacc_add(kl->tacc, isprop ? 1 : 0, conf, (double)sumsq);
  }
  if constexpr (!PREP && !SPL) {   // SPL: wave 1 made them
    if (!isprop) walker_draws<T, N>(kl, conf, lane);
  }
  AQ_PH(9);
}

}  // namespace aq
