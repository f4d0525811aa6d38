// jets.h -- per-lane Taylor jets and wave primitives for the AIQMC walker kernels.
//
// Lane layout of one 64-wide wavefront that evaluates ONE electron
// configuration (N <= 16 electrons):
//
//   lane l = 16*c + e      c = l >> 4 in {0,1,2,3},  e = l & 15
//   c < 3, e < N : "direction lane" for the coordinate x_{e,c}
//   c == 3       : "value row" (lanes 48..63)
//
// PJ<T>  {v, d1, d2}: every lane carries a value and the first/second
//        derivative along its OWN direction (value-row lanes: direction 0).
//        Used for per-electron and per-pair streams, whose values differ
//        between lanes.
// DJ<T>  {d1, d2}: a quantity shared by the whole wave.  Direction lanes hold
//        the first/second directional derivative; value-row lanes hold the
//        value in d1.  One VGPR (two with second derivatives) per scalar.
//
// The second derivative kept per lane is the diagonal Hessian entry along the
// lane's coordinate, so the Laplacian is the sum over direction lanes (the
// forward-Laplacian of the reference's jvp-of-grad loop,
// Energy/hamiltonian.py:100-131).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aq {

// Pointer to the packed kernel parameters (and other per-wave-uniform tables): the constant
// address space, so that reads at wave-uniform offsets become scalar loads through the
// scalar cache (s_load / s_buffer_load) instead of vector-memory instructions; reads at
// per-lane offsets stay vector loads.  Measured on the N2 proposal launch: 310 -> 296 us
// (fewer VMEM instructions outweigh the extra v_mov the one-SGPR VOP3 operand rule costs).
template <typename T> using cptr = const __attribute__((address_space(4))) T* __restrict__;
template <typename T> __device__ __forceinline__ cptr<T> param_ptr(const void* p) {
  return (cptr<T>)(const __attribute__((address_space(4))) void*)p;
}

// Scalar math.  float uses the hardware approximations (v_sqrt_f32, v_rcp_f32,
// v_exp_f32: ~1 ulp), which is well inside the fp32 parity tolerance of the
// reference's own float32 arithmetic; double keeps the correctly rounded
// library functions (the fp64 parity mode).
template <typename T> __device__ __forceinline__ T f_sqrt(T x);
template <> __device__ __forceinline__ float f_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
template <> __device__ __forceinline__ double f_sqrt(double x) { return sqrt(x); }
template <typename T> __device__ __forceinline__ T f_rcp(T x);
template <> __device__ __forceinline__ float f_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
template <> __device__ __forceinline__ double f_rcp(double x) { return 1.0 / x; }
template <typename T> __device__ __forceinline__ T f_div(T a, T b);
template <> __device__ __forceinline__ float f_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
template <> __device__ __forceinline__ double f_div(double a, double b) { return a / b; }
template <typename T> __device__ __forceinline__ T f_exp(T x);
template <> __device__ __forceinline__ float f_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
template <> __device__ __forceinline__ double f_exp(double x) { return exp(x); }
template <typename T> __device__ __forceinline__ T f_log(T x);
template <> __device__ __forceinline__ float f_log(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
template <> __device__ __forceinline__ double f_log(double x) { return log(x); }
// tanh(x) = 1 - 2/(1 + e^{2x}); saturates correctly at +-inf (abs. error ~1e-7 in float)
template <typename T> __device__ __forceinline__ T f_tanh(T x);
template <> __device__ __forceinline__ float f_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + e);
}
template <> __device__ __forceinline__ double f_tanh(double x) { return tanh(x); }
// mantissa in [0.5, 1) and binary exponent (v_frexp_mant / v_frexp_exp)
__device__ __forceinline__ float f_frexp(float x, int& e) { return frexpf(x, &e); }
__device__ __forceinline__ double f_frexp(double x, int& e) { return frexp(x, &e); }
__device__ __forceinline__ float f_ldexp(float x, int e) { return ldexpf(x, e); }
__device__ __forceinline__ double f_ldexp(double x, int e) { return ldexp(x, e); }
template <typename T> __device__ __forceinline__ T f_abs(T x);
template <> __device__ __forceinline__ float f_abs(float x) { return fabsf(x); }
template <> __device__ __forceinline__ double f_abs(double x) { return fabs(x); }

// 1 / pivot (ir, ii), 1 / |pivot| (rabs) and |pivot|^2 = m 2^e (m in [1/2, 1), frexp form) of a
// complex pivot pr + i pim, den = pr^2 + pim^2 already formed.  den leaves the floating-point range
// on both sides for a row scaled by a far-out electron's envelope: fp32 below |pivot| ~ 1e-15 (a
// Gaussian envelope ~1e-19: 1 / den overflows, inf - inf turns the inverse into NaN; below ~1e-23
// den itself underflows to 0 and log|det| is -inf) and above |pivot| ~ 1e15 (the signed
// exp(-pi ae) term of envelope.py:29-30, ~1e21 at 50 bohr: den overflows, 1 / pivot becomes 0).
// That (rare, wave-uniform in the Gauss-Jordan) case scales the pivot by the power of two of its
// larger component first, so every quantity is formed in range, exactly as jnp.linalg.slogdet's
// scaled pivots stay finite (network_blocks.py:156).  Ordinary pivots take the plain formulas,
// bit for bit as before.
template <typename T> struct PivRange;
template <> struct PivRange<float> { static constexpr float lo = 1e-30f, hi = 1e30f; };
template <> struct PivRange<double> { static constexpr double lo = 1e-290, hi = 1e290; };
template <typename T>
__device__ __forceinline__ void pivot_recip_me(T pr, T pim, T den, T& ir, T& ii, T& rabs, T& m, int& e) {
  if (!(den >= PivRange<T>::lo && den <= PivRange<T>::hi)) {
    const T s = f_abs(pr) > f_abs(pim) ? f_abs(pr) : f_abs(pim);
    int es;
    (void)f_frexp(s, es);
    const T a = f_ldexp(pr, -es), b = f_ldexp(pim, -es);   // exact: |a|, |b| < 1
    const T d1 = a * a + b * b;                              // in [1/4, 2)
    const T rd = f_rcp(d1);
    ir = f_ldexp(a * rd, -es);
    ii = f_ldexp(-b * rd, -es);
    rabs = f_ldexp(f_sqrt(rd), -es);
    int e1;
    m = f_frexp(d1, e1);
    e = e1 + 2 * es;
  } else {
    const T rden = f_rcp(den);
    ir = pr * rden;
    ii = -pim * rden;
    rabs = f_sqrt(rden);
    m = f_frexp(den, e);
  }
}
// |pivot|^2 = m 2^e (m in [1/2, 1)) for any finite pivot, branch-free.  float: the square formed
// in double (exact products, one rounding; no float pivot leaves double's range); double: the
// pivot scaled by the power of two of its larger component first (exact scalings).
__device__ __forceinline__ float pivot_mag2(float pr, float pim, int& e) {
  const double a = (double)pr, b = (double)pim;
  return (float)frexp(a * a + b * b, &e);
}
__device__ __forceinline__ double pivot_mag2(double pr, double pim, int& e) {
  int es, e1;
  (void)frexp(fabs(pr) > fabs(pim) ? fabs(pr) : fabs(pim), &es);
  const double a = ldexp(pr, -es), b = ldexp(pim, -es);
  const double m = frexp(a * a + b * b, &e1);
  e = e1 + 2 * es;
  return m;
}
// the same with log |pivot|^2 (lden) instead of the frexp form
template <typename T>
__device__ __forceinline__ void pivot_recip(T pr, T pim, T den, T& ir, T& ii, T& rabs, T& lden) {
  if (!(den >= PivRange<T>::lo && den <= PivRange<T>::hi)) {
    T m;
    int e;
    pivot_recip_me(pr, pim, den, ir, ii, rabs, m, e);
    lden = f_log(m) + T(e) * T(0.69314718055994531);
  } else {
    const T rden = f_rcp(den);
    ir = pr * rden;
    ii = -pim * rden;
    rabs = f_sqrt(rden);
    lden = f_log(den);
  }
}
__device__ __forceinline__ float f_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double f_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
template <typename T> __device__ __forceinline__ T f_hypot(T x, T y);
template <> __device__ __forceinline__ float f_hypot(float x, float y) { return hypotf(x, y); }
template <> __device__ __forceinline__ double f_hypot(double x, double y) { return hypot(x, y); }
template <typename T> __device__ __forceinline__ T f_atan2(T y, T x);
template <> __device__ __forceinline__ float f_atan2(float y, float x) { return atan2f(y, x); }
template <> __device__ __forceinline__ double f_atan2(double y, double x) { return atan2(y, x); }

// ---------------------------------------------------------------------------
// PJ: univariate second-order Taylor jet along the lane's direction
// ---------------------------------------------------------------------------
template <typename T> struct PJ { T v, d1, d2; };

template <typename T> __device__ __forceinline__ PJ<T> pjc(T c) { return PJ<T>{c, T(0), T(0)}; }
template <typename T> __device__ __forceinline__ PJ<T> operator+(PJ<T> a, PJ<T> b) {
  return PJ<T>{a.v + b.v, a.d1 + b.d1, a.d2 + b.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator-(PJ<T> a, PJ<T> b) {
  return PJ<T>{a.v - b.v, a.d1 - b.d1, a.d2 - b.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator-(PJ<T> a) {
  return PJ<T>{-a.v, -a.d1, -a.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator*(PJ<T> a, PJ<T> b) {
  return PJ<T>{a.v * b.v, a.d1 * b.v + a.v * b.d1, a.d2 * b.v + T(2) * a.d1 * b.d1 + a.v * b.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator*(T s, PJ<T> a) {
  return PJ<T>{s * a.v, s * a.d1, s * a.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator*(PJ<T> a, T s) {
  return PJ<T>{s * a.v, s * a.d1, s * a.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator+(PJ<T> a, T s) {
  return PJ<T>{a.v + s, a.d1, a.d2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator-(PJ<T> a, T s) {
  return PJ<T>{a.v - s, a.d1, a.d2};
}
// a / b   (a = q b  =>  q' = (a' - q b')/b,  q'' = (a'' - 2 q' b' - q b'')/b)
template <typename T> __device__ __forceinline__ PJ<T> operator/(PJ<T> a, PJ<T> b) {
  const T ib = f_rcp(b.v);
  const T q = f_div(a.v, b.v);
  const T q1 = (a.d1 - q * b.d1) * ib;
  const T q2 = (a.d2 - T(2) * q1 * b.d1 - q * b.d2) * ib;
  return PJ<T>{q, q1, q2};
}
template <typename T> __device__ __forceinline__ PJ<T> operator/(PJ<T> a, T s) {
  const T is = f_rcp(s);
  return PJ<T>{f_div(a.v, s), a.d1 * is, a.d2 * is};
}
template <typename T> __device__ __forceinline__ PJ<T> pj_sqrt(PJ<T> a) {
  const T s = f_sqrt(a.v);
  const T h = T(0.5) * f_rcp(s);
  const T s1 = a.d1 * h;
  return PJ<T>{s, s1, (a.d2 - T(2) * s1 * s1) * h};
}
template <typename T> __device__ __forceinline__ PJ<T> pj_exp(PJ<T> a) {
  const T e = f_exp(a.v);
  return PJ<T>{e, e * a.d1, e * (a.d2 + a.d1 * a.d1)};
}
template <typename T> __device__ __forceinline__ PJ<T> pj_tanh(PJ<T> a) {
  const T t = f_tanh(a.v);
  const T s = T(1) - t * t;
  return PJ<T>{t, s * a.d1, s * a.d2 - T(2) * t * s * a.d1 * a.d1};
}
template <typename T> __device__ __forceinline__ PJ<T> pj_sel(bool c, PJ<T> a, PJ<T> b) {
  return PJ<T>{c ? a.v : b.v, c ? a.d1 : b.d1, c ? a.d2 : b.d2};
}

// ---------------------------------------------------------------------------
// wave primitives
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rdlane(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
__device__ __forceinline__ double rdlane(double x, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ int rdlane(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// Every DPP pattern used here (quad_perm, row_ror, row_mirror, row_newbcast) has a
// valid source lane for every lane, so bound_ctrl is set and no "old" value is needed;
// this lets the compiler fold the move into the consuming VOP2 instruction.
template <int CTRL> __device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int CTRL> __device__ __forceinline__ double dpp(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, true);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Sum over the 16 lanes of each DPP row; every lane of the row receives the
// (bitwise identical) row total.  quad_perm[1,0,3,2], quad_perm[2,3,0,1],
// row_half_mirror, row_mirror.
template <typename T> __device__ __forceinline__ T rowsum16(T x) {
  x += dpp<0xB1>(x);
  x += dpp<0x4E>(x);
  x += dpp<0x141>(x);
  x += dpp<0x140>(x);
  return x;
}

// K independent row sums, interleaved so the DPP read-after-write hazards overlap.
template <typename T, int K> __device__ __forceinline__ void rowsum16_multi(T* x) {
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] += dpp<0xB1>(x[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] += dpp<0x4E>(x[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] += dpp<0x141>(x[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] += dpp<0x140>(x[k]);
}

// Sum over all 64 lanes, uniform result.
template <typename T> __device__ __forceinline__ T wave_sum(T x) {
  x = rowsum16(x);
  return (rdlane(x, 0) + rdlane(x, 16)) + (rdlane(x, 32) + rdlane(x, 48));
}

// ---------------------------------------------------------------------------
// Pair<T>: two values in adjacent registers.  fp32 uses a 2-vector so that the
// backend issues packed VOP3P math (v_pk_fma_f32 / v_pk_mul_f32: two FMAs per
// instruction, op_sel broadcasting a scalar operand); fp64 has no packed math.
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
struct D2 { double x, y; };
template <typename T> struct Pair;
template <> struct Pair<float> { using type = f32x2; };
template <> struct Pair<double> { using type = D2; };
template <typename T> __device__ __forceinline__ typename Pair<T>::type pair_make(T a, T b);
template <> __device__ __forceinline__ f32x2 pair_make<float>(float a, float b) { return f32x2{a, b}; }
template <> __device__ __forceinline__ D2 pair_make<double>(double a, double b) { return D2{a, b}; }
template <typename T> __device__ __forceinline__ T pair_re(typename Pair<T>::type v) { return v.x; }
template <typename T> __device__ __forceinline__ T pair_im(typename Pair<T>::type v) { return v.y; }
// s * v
template <typename T> __device__ __forceinline__ typename Pair<T>::type pair_scale(typename Pair<T>::type v, T s);
template <> __device__ __forceinline__ f32x2 pair_scale<float>(f32x2 v, float s) { return v * f32x2{s, s}; }
template <> __device__ __forceinline__ D2 pair_scale<double>(D2 v, double s) { return D2{v.x * s, v.y * s}; }
// s * v + w
template <typename T>
__device__ __forceinline__ typename Pair<T>::type pair_fma(T s, typename Pair<T>::type v, typename Pair<T>::type w);
template <> __device__ __forceinline__ f32x2 pair_fma<float>(float s, f32x2 v, f32x2 w) {
  return __builtin_elementwise_fma(f32x2{s, s}, v, w);
}
template <> __device__ __forceinline__ D2 pair_fma<double>(double s, D2 v, D2 w) {
  return D2{__builtin_fma(s, v.x, w.x), __builtin_fma(s, v.y, w.y)};
}

// ---------------------------------------------------------------------------
// DJ: wave-shared jet (direction lanes: derivatives, value row: value in d1)
// ---------------------------------------------------------------------------
template <typename T> struct DJ { T d1, d2; };

template <typename T> __device__ __forceinline__ DJ<T> dj_zero() { return DJ<T>{T(0), T(0)}; }
template <typename T> __device__ __forceinline__ void dj_axpy(DJ<T>& acc, T w, DJ<T> x) {
  acc.d1 += w * x.d1;
  acc.d2 += w * x.d2;
}
// tanh of a wave-shared jet; the value is broadcast from lane 48.
template <typename T> __device__ __forceinline__ DJ<T> dj_tanh(DJ<T> z, bool val) {
  const T zv = rdlane(z.d1, 48);
  const T t = f_tanh(zv);
  const T s = T(1) - t * t;
  DJ<T> o;
  o.d1 = val ? t : s * z.d1;
  o.d2 = s * z.d2 - T(2) * t * s * z.d1 * z.d1;
  return o;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (production random draws)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// 4 uniforms from (seed, step, stream id, kind): u in (0,1] (24-bit grid)
__device__ __forceinline__ void philox_u4(uint64_t seed, uint64_t step, uint32_t sid, uint32_t kind, float u[4]) {
  uint32_t c[4] = {sid, (uint32_t)step, (uint32_t)(step >> 32), kind};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = (float)((c[j] >> 8) + 1u) * 5.9604644775390625e-08f;
}
// 3 standard normals (Box-Muller on 4 uniforms, float math)
__device__ __forceinline__ void philox_normal3f(uint64_t seed, uint64_t step, uint32_t sid, uint32_t kind,
                                                float out[3]) {
  float u[4];
  philox_u4(seed, step, sid, kind, u);
  const float r0 = sqrtf(-2.0f * __logf(u[0])), r1 = sqrtf(-2.0f * __logf(u[2]));
  float s0, c0, s1, c1;
  __sincosf(6.283185307179586f * u[1], &s0, &c0);
  __sincosf(6.283185307179586f * u[3], &s1, &c1);
  out[0] = r0 * c0;
  out[1] = r0 * s0;
  out[2] = r1 * c1;
}

}  // namespace aq
