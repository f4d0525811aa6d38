// valu_rate.hip -- microbenchmark: VALU issue rate on gfx950 for the instruction kinds the
// walker kernels are made of (plain f32 FMA, FMA with a DPP-broadcast operand, v_exp_f32,
// packed v_pk_fma_f32, ds_swizzle-free DPP row sums), at 1..8 waves per SIMD.
// Prints cycles per wave-instruction per SIMD = (wave lifetime cycles) / (waves/SIMD * insts).
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ITERS = 2048;
constexpr int ILP = 8;

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(64) void k_rate(float* out, unsigned long long* cyc, float a, float b) {
  float x[ILP];
  f2 p[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) {
    x[k] = threadIdx.x * 0.001f + k;
    p[k] = f2{x[k], x[k] + 1.f};
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      if constexpr (KIND == 0) {          // v_fma_f32
        x[k] = __builtin_fmaf(x[k], a, b);
      } else if constexpr (KIND == 1) {   // v_fmac_f32 with a DPP row_newbcast operand
        const float d = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x[(k + 1) % ILP]), 0x153, 0xF, 0xF, true));
        x[k] = __builtin_fmaf(d, a, x[k]);
      } else if constexpr (KIND == 2) {   // v_exp_f32
        x[k] = __builtin_amdgcn_exp2f(x[k]);
      } else if constexpr (KIND == 3) {   // v_pk_fma_f32
        p[k] = __builtin_elementwise_fma(p[k], f2{a, a}, f2{b, b});
      } else if constexpr (KIND == 4) {   // v_add_f32 with a quad_perm DPP operand (quad sums)
        x[k] += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x[k]), 0xB1, 0xF, 0xF, true));
      } else if constexpr (KIND == 5) {   // v_rcp_f32
        x[k] = __builtin_amdgcn_rcpf(x[k]);
      } else if constexpr (KIND == 6) {   // v_cndmask_b32 (select on a lane-dependent compare)
        x[k] = (x[k] > b) ? x[k] : x[(k + 3) % ILP];
      } else if constexpr (KIND == 7) {   // v_mov_b32_dpp row_newbcast alone (result used by a plain add)
        const float d = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x[(k + 1) % ILP]), 0x153, 0xF, 0xF, false));
        x[k] = x[k] + d;
      } else if constexpr (KIND == 8) {   // integer v_add_u32 + v_lshl_add_u32 (address-style arithmetic)
        int v = __builtin_bit_cast(int, x[k]);
        v = (v << 2) + (int)threadIdx.x;
        x[k] = __builtin_bit_cast(float, v);
      } else if constexpr (KIND == 9) {   // v_readlane_b32 to an SGPR and back into a VALU op
        x[k] = x[k] + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x[(k + 1) % ILP]), k));
      }
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += x[k] + p[k].x + p[k].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, int waves_per_simd) {
  const int nblk = 256 * 4 * waves_per_simd;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)nblk * 64 * 4);
  hipMalloc(&cyc, (size_t)nblk * 8);
  k_rate<KIND><<<nblk, 64>>>(out, cyc, 1.0001f, 0.5f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k_rate<KIND><<<nblk, 64>>>(out, cyc, 1.0001f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(nblk);
  hipMemcpy(h.data(), cyc, nblk * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : h) avg += (double)v;
  avg /= nblk;
  const double insts = (double)ITERS * ILP * ((KIND == 1 || KIND == 4 || KIND == 6 || KIND == 7 || KIND == 9) ? 2 : 1);
  printf("%-12s waves/SIMD=%d  wave cycles=%.0f  cyc/inst/SIMD=%.2f  wall=%.3f ms  clk=%.2f GHz\n", name,
         waves_per_simd, avg, avg / (waves_per_simd * insts), ms, avg / (ms * 1e6));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {1, 2, 4, 5, 8}) {
    run<0>("fma", w);
    run<1>("fma+dpp", w);
    run<4>("add+dpp", w);
    run<2>("exp", w);
    run<5>("rcp", w);
    run<3>("pk_fma", w);
    run<6>("cndmask", w);
    run<7>("dppmov+add", w);
    run<8>("int2", w);
    run<9>("readlane+add", w);
  }
  return 0;
}
