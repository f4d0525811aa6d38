// ctx.h -- host-side context + per-shape dispatch table shared by the
// C-ABI translation unit (aiqmc.hip) and the per-shape kernel TUs (shape.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "aiqmc.h"
#include "walker_kernel.h"

int aiqmc_fail(int code, const std::string& msg);
using aq::KArgs;
#include <utility>
#define AIQMC_PROF_SLOTS 4

struct aiqmc_ctx {
  int N = 0, A = 0, nup = 0, ndn = 0, dtype = 0, device = 0;
  int npar = 0, nanti = 0;
  std::vector<double> atoms, charges;
  std::vector<int> up, dn, par, anti;
  int64_t ncanon = 0, nkern = 0, nprm = 0;   // nprm: device parameter buffer (nkern + lane-order copies)
  void* d_prm = nullptr;
  int* d_rowsrc = nullptr;
  bool params_set = false;
  int ws_B = 0;
  void *d_grad = nullptr, *d_lp = nullptr, *d_sq = nullptr, *d_lpn = nullptr, *d_gown = nullptr,
       *d_sqn = nullptr;
  void *d_g1 = nullptr, *d_g2 = nullptr, *d_u = nullptr;   // per-sweep Philox draws
  void *d_wc = nullptr, *d_ec = nullptr;                    // Metropolis caches (walker_rev.h WCache/ECache)
  void* d_wcp = nullptr;                                    // per-proposal cache scratch (reuse off)
  int64_t wcp_n = 0;                                        // its capacity in configurations
  void* d_lc = nullptr;                                     // local-energy LapCache [B][lcache_n]
  int lc_B = 0, lc_n = 0;
  void* d_cx = nullptr;                                     // complex E_L scratch [B][6N+1]: grad log|psi|, grad theta, lap theta
  int cx_B = 0;
  bool reuse = true;                                        // proposals reuse the walker's cached stage
  int ablate = 0;                                           // AQ_ABLATE development builds (walker_rev.h)
  int fuse_accept = 1;                                      // acceptance fused into the next walker launch
  int walker_fixed_gj = 1;                                  // walker launches re-use the previous sweep's pivot order
  int quad_pivoted = 0;                                     // k_quad_value: partial pivoting for every slot (test)
  int packed_walkers = 1;                                   // N <= 8 walker launches several per wave
  int fuse_reduce = 1;                                      // fp32 mc_step: limdrift sums by integer atomics
  int wide_reduce = 1;                                      // unfused fp32 sweeps: k_taueff_part (0: k_taueff)
  unsigned long long* d_tpart = nullptr;                    // their per-sweep partial sums [tpart_n][2][TPART]
  int tpart_n = 0;
  unsigned long long* d_tacc = nullptr;                     // their per-sweep accumulators [2 banks][tacc_n][2]
  int tacc_n = 0;
  int tacc_bank = 0;                                        // the bank the next mc_step call uses
  bool tacc_clean[2] = {false, false};                      // bank zeroed (by the last k_accept of a call)
  int lap_waves = 0;                                        // waves per walker of k_walker_lap (0: by batch)
  int ncu = 256;                                            // compute units of the device
  double* d_taueff = nullptr;
  int64_t ws_bytes = 0;
  // pseudopotential (aiqmc_set_ecp / aiqmc_local_energy_ecp, ecp.h)
  bool ecp_set = false;
  int ecp_KL = 0, ecp_KN = 0, ecp_L = 0;
  bool ecp_nl_zero = false;   // every nonlocal coefficient 0 (all-electron through the pp path)
  double* d_ecp_tab = nullptr;
  int ecp_B = 0;
  void *d_ecp_rot = nullptr, *d_ecp_x = nullptr, *d_ecp_lq = nullptr, *d_ecp_pq = nullptr, *d_ecp_ec = nullptr,
       *d_ecp_el = nullptr, *d_ecp_lp0 = nullptr, *d_ecp_ph0 = nullptr;
  int64_t ecp_bytes = 0;
  double* d_tm_scr = nullptr;      // T-moves per-walker amplitudes [tm_B][N*A*50][4]
  double* d_dscr = nullptr;        // DMC reduction scratch: block partial sums / cut minima [2*64]
  int tm_B = 0;
  // parameter gradients (aiqmc_logpsi_param_grad, walker_pgrad.h)
  int* d_gmap = nullptr;            // [ncanon]
  double* d_wnorm = nullptr;        // [6] |W_y row| of the current parameters
  // device repack program of aiqmc_set_params_device (built once per context from pack_params):
  // per kernel-layout entry an op (0 constant, 1 copy, 2 row-normalised y coefficient), its
  // canonical source index and its constant value
  int* d_pk_op = nullptr;
  int* d_pk_src = nullptr;
  double* d_pk_cval = nullptr;
  void* d_pg = nullptr;             // [pg_B][nkern] per-walker kernel-layout gradients
  void* d_pgr = nullptr;            // [nkern] weighted sum
  int pg_B = 0;
  int pg_nw = 0;                     // weighted rows d_pgr holds before its chunk sums
  // optional per-kernel HIP-event timing (aiqmc_profile_*): slot -> recorded (start, stop) pairs
  bool prof = false;
  std::vector<hipEvent_t> ev_free;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used[AIQMC_PROF_SLOTS];
};

struct ShapeOps {
  int (*set_lds)();
  void (*walker)(int dtype, int mode, const KArgs& ka, int nconf, hipStream_t s);
  void (*accept)(int dtype, void* pos, const aq::AccArgs& a, int B, hipStream_t s);
  void (*moved)(int dtype, const KArgs& ka, hipStream_t s);   // k_moved_electron over ka.nconf proposals
  // local energy: adjoint pass (k1) + first-derivative pass (k2), walker_lap.h
  void (*lap)(int dtype, const KArgs& k1, const KArgs& k2, int nconf, int waves, int phase, hipStream_t s);
  void (*phase_read)(unsigned long long* out32);               // AQ_PHASE_PROF builds only
  int wcache_n, ecache_n;                                      // cache entries per walker / per proposal
  int lcache_n;                                                // LapCache entries per walker
  int64_t nkern;
  int64_t nprm;
  long (*ncanon)(int npar, int nanti);
  void (*pack)(const aiqmc_ctx* c, const double* flat, std::vector<double>& out);
  void (*gmap)(const aiqmc_ctx* c, std::vector<int>& map);                        // canonical -> kernel index
  int (*pgrad)(int dtype, const KArgs& ka, int nconf, hipStream_t s);            // k_param_grad
  int wy_off;                                                                      // Lay::wy
  // dynamic LDS bytes per workgroup of the launches that take it, [dtype f32, f64][kind]
  // (kind: AIQMC_LDS_* of aiqmc.h), and the waves per workgroup of each: what a profiler's
  // dispatch record does not show (rocprofv3 reports the static group segment only)
  int dyn_lds[2][6];
  int wg_waves[2][6];
};


