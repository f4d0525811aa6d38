/*
 * aiqmc.h -- C-ABI of the MI355X-native AIQMC VMC inner loop.
 *
 * The reference (Yongda1/AIQMC, AIQMCrelease3) is pure Python/JAX and has no
 * FFI; the entry points below replace the JAX-traced hot path one for one:
 *
 *   aiqmc_logpsi        <- network.apply / signed_network, vmapped
 *                          (AIQMCrelease3/wavefunction_Ynlm/nn.py:545-551,
 *                           network_blocks.py:161-206)
 *   aiqmc_logpsi_grad   <- vmap(jax.grad(logabs_f))   (VMC/VMCmcstep.py:41-53)
 *   aiqmc_local_energy  <- vmap(hamiltonian.local_energy(...)) with
 *                          complex_output=False (Energy/hamiltonian.py:236-260,
 *                          kinetic part :77-132)
 *   aiqmc_mc_step       <- VMCmcstep.main_monte_carlo(...) -> mc_step
 *                          (VMC/VMCmcstep.py:121-140, walkers_update :28-111)
 *   aiqmc_set_params    <- the params pytree passed to all of the above;
 *                          `flat` is its jax.tree_util.tree_flatten order
 *                          (dict keys sorted, lists in order, C-order leaves),
 *                          i.e. jax.flatten_util.ravel_pytree(params)[0].
 *
 * Conventions: every array pointer passed to a compute entry point is a DEVICE
 * pointer (HIP) of the context's dtype (float for AIQMC_F32, double for
 * AIQMC_F64); `stream` is a hipStream_t (NULL = default stream).  Host
 * pointers appear only in aiqmc_cfg and aiqmc_set_params.  Functions return
 * 0 on success and a negative AIQMC_E* code on failure; the message is in
 * aiqmc_last_error() (thread-local).  No C++ exception crosses the ABI.
 * A context is bound to one device and is not re-entrant.
 */
#ifndef AIQMC_H_
#define AIQMC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIQMC_F32 0
#define AIQMC_F64 1

#define AIQMC_OK 0
#define AIQMC_EINVAL (-1)
#define AIQMC_EUNSUPPORTED (-2)
#define AIQMC_EHIP (-3)
#define AIQMC_ESTATE (-4)

/* rng_mode of aiqmc_mc_step */
#define AIQMC_RNG_HOST 0    /* gauss1/gauss2/u supplied by the caller (parity mode) */
#define AIQMC_RNG_PHILOX 1  /* drawn on device from (seed, offset)                 */

typedef struct aiqmc_ctx aiqmc_ctx;

/* System + network configuration (make_ai_net arguments, nn.py:511-526). */
typedef struct aiqmc_cfg {
  int32_t nelectrons;            /* N  (2 <= N <= 16)                          */
  int32_t natoms;                /* A  ((N, A) in aiqmc_supported_shapes():   */
                                 /*     every N with A <= 3, and (10,4),(10,5)) */
  int32_t nspins[2];             /* (n_up, n_down); both > 0                   */
  int32_t dtype;                 /* AIQMC_F32 | AIQMC_F64                      */
  int32_t device;                /* HIP device ordinal                         */
  const double* atoms;           /* [A*3] bohr                                 */
  const double* charges;         /* [A]   (Jastrow e-n + potential charges)    */
  const int32_t* spin_up_indices;   /* [n_up]   spin_indices.py:38-45          */
  const int32_t* spin_down_indices; /* [n_down]                                */
  const int32_t* parallel_indices;  /* [2*n_parallel] row-major (2,n_par)      */
  int32_t n_parallel;               /* spin_indices.py:5-19                    */
  const int32_t* antiparallel_indices; /* [2*n_antiparallel]                   */
  int32_t n_antiparallel;
  int32_t hidden_dims[3][2];     /* must be ((4,4),(4,4),(4,4)) (nn.py:525)   */
  int32_t hidden_dims_ynlm[3];   /* must be (6,6,6)             (nn.py:526)   */
} aiqmc_cfg;

int aiqmc_create(const aiqmc_cfg* cfg, aiqmc_ctx** out);
int aiqmc_destroy(aiqmc_ctx* ctx);

/* Number of doubles aiqmc_set_params expects (2381 for N2 with defaults). */
int64_t aiqmc_param_count(const aiqmc_ctx* ctx);

/* flat: HOST pointer, `n` doubles in tree_flatten order. Synchronous upload. */
int aiqmc_set_params(aiqmc_ctx* ctx, const double* flat, int64_t n, void* stream);

/* flat: DEVICE pointer (this context's device), `n` doubles in tree_flatten order, repacked into
 * the kernel layout on `stream` (stream-ordered, no host synchronisation): the parameters of an
 * optimiser step that stays on the device (the reference's params are device arrays updated by
 * optax / kfac inside pmap, adam.py:49-59).  The kernel layout equals aiqmc_set_params' bitwise. */
int aiqmc_set_params_device(aiqmc_ctx* ctx, const double* flat, int64_t n, void* stream);

/* pos[B*3N] -> logabs[B], phase[B] (phase may be NULL). */
int aiqmc_logpsi(aiqmc_ctx* ctx, const void* pos, int32_t B, void* logabs, void* phase,
                 void* stream);

/* pos[B*3N] -> logabs[B] (may be NULL), grad[B*3N] = d log|psi| / d pos. */
int aiqmc_logpsi_grad(aiqmc_ctx* ctx, const void* pos, int32_t B, void* logabs, void* grad,
                      void* stream);

/* pos[B*3N] -> e_l[B]; logabs[B] and grad[B*3N] optional (NULL to skip). */
int aiqmc_local_energy(aiqmc_ctx* ctx, const void* pos, int32_t B, void* e_l, void* logabs,
                       void* grad, void* stream);

/* complex_output=True local energy (replaces Energy/hamiltonian.py:100-131 with complex_output
 * True, i.e. local_kinetic_energy's phase branch :110-130, + the potential :236-260):
 * pos[B*3N] -> e_re[B], e_im[B] with
 *   KE = -1/2 [lap log|psi| + i lap theta] - 1/2 |grad log|psi||^2 + 1/2 |grad theta|^2
 *        - i grad log|psi| . grad theta,   theta = arg psi,
 * E_L = V + KE.  Two local-energy launch pairs (log|psi| and theta) and one combining launch. */
int aiqmc_local_energy_complex(aiqmc_ctx* ctx, const void* pos, int32_t B, void* e_re, void* e_im,
                               void* stream);

/* nsteps drift-diffusion Metropolis steps on pos_inout[B*3N] (in place; the
 * donate_argnums=1 analogue).  B is the per-device batch: limdrift's v2 is
 * summed over exactly these B walkers (VMCmcstep.py:12).
 * AIQMC_RNG_HOST: gauss1[nsteps*B*3N] and gauss2[nsteps*B*N*3] standard
 * normals (gauss2 = the electron-diagonal blocks of the reference's
 * [B,N,3N] draw, the only entries it reads, VMCmcstep.py:87-94) and
 * u[nsteps*B*N] uniforms in [0,1).  AIQMC_RNG_PHILOX: the three may be NULL;
 * draws come from Philox4x32-10 keyed by seed, counter offset+step.
 * accept_out (optional, int32[B]) accumulates accepted single-electron moves. */
int aiqmc_mc_step(aiqmc_ctx* ctx, void* pos_inout, int32_t B, int32_t nsteps, double tstep,
                  int32_t rng_mode, const void* gauss1, const void* gauss2, const void* u,
                  uint64_t seed, uint64_t offset, int32_t* accept_out, void* stream);

/* Parameter gradient of log|psi| (the psi_tangent of the energy-gradient custom JVP,
 * Loss/loss.py:242-265, differentiated wrt params as jax.value_and_grad does in
 * Optimizer/adam.py:51-54).  Output in the canonical tree_flatten order of
 * aiqmc_set_params (aiqmc_param_count entries; unused leaves eplion/mu/nu get 0):
 *   weights == NULL: out[B][P] = d log|psi(x_b)| / d theta      (per walker)
 *   weights != NULL: out[P]    = sum_b weights[b] d log|psi(x_b)| / d theta
 * weights/out/logabs are device arrays of the context dtype; logabs[B] optional. */
int aiqmc_logpsi_param_grad(aiqmc_ctx* ctx, const void* pos, int32_t B, const void* weights, void* out,
                            void* logabs, void* stream);

/* Parameter gradient of the phase of psi (arg det A; the Jastrows are real), the imaginary
 * part of psi_tangent when the driver differentiates the complex log
 * log|psi| + i phase (Loss/loss.py:256-265 with complex_output=True, network = log_network
 * of main_pp_adam_muti_GPU.py:119-121).  Same layout and weights convention as
 * aiqmc_logpsi_param_grad; phase[B] (optional) receives the phase at the walkers. */
int aiqmc_phase_param_grad(aiqmc_ctx* ctx, const void* pos, int32_t B, const void* weights, void* out,
                           void* phase, void* stream);

/* Several weighted sums from ONE per-walker gradient pass: out[k][P] = sum_b weights[k][b]
 * d f(x_b) / d theta for k < nw (1..8), f = log|psi| (phase == 0) or the phase (phase != 0);
 * vals[B] (optional) receives f at the walkers.  (The multi-rank energy gradient needs the
 * clipping-weighted sum and the plain sum of d log|psi| together, aiqmc_loss_level.) */
int aiqmc_param_grad_weighted(aiqmc_ctx* ctx, const void* pos, int32_t B, int32_t phase, const void* weights,
                              int32_t nw, void* out, void* vals, void* stream);

/* The orbital matrix of B walkers (Network.orbitals = make_orbitals.apply, nn.py:409-506,553):
 * orbitals[B][N][N][2] (re, im; ctx dtype) = Phi * Yt * exp(J_ee/N) exp(J_ae/N), rows = up
 * electrons then down electrons (spin_up_indices / spin_down_indices order), row r's envelope
 * and y row those of electron r (quirk Q1).  logabs / phase (optional, [B]) as aiqmc_logpsi. */
int aiqmc_orbitals(aiqmc_ctx* ctx, const void* pos, int32_t B, void* orbitals, void* logabs, void* phase,
                   void* stream);

/* DMC drift-diffusion step (DMC/drift_diffusion.py:25-107): one Metropolis sweep
 * exactly as aiqmc_mc_step with nsteps = 1 (same draws, in place), plus
 *   grad_eff_old[B*3N]  limdrift(grad log|psi|) at the walkers before the move (:60-61),
 *   grad_new_eff[B*3N]  limdrift(grad log|psi|) at the moved walkers (:103-104),
 *   tdamp[3]            device doubles: [sum of proposed coordinates, sum of new
 *                       coordinates, tdamp = their ratio] (walkers_accept :21). */
int aiqmc_dmc_drift_diffusion(aiqmc_ctx* ctx, void* pos_inout, int32_t B, double tstep, int32_t rng_mode,
                              const void* gauss1, const void* gauss2, const void* u, uint64_t seed, uint64_t offset,
                              void* grad_eff_old, void* grad_new_eff, double* tdamp, void* stream);

/* DMC weight update (DMC/S_matrix.py:4-24, dmc.py:80-92): with S from the real
 * local energies eloc_old/eloc_new [B], v2 = |grad_eff|^2 per walker and the tdamp[3]
 * array of aiqmc_dmc_drift_diffusion (its entry 2 is used),
 * weights[B] *= exp(tstep tdamp (S_new + S_old)/2). */
int aiqmc_dmc_weights(aiqmc_ctx* ctx, int32_t B, const void* eloc_old, const void* eloc_new, const void* grad_eff_old,
                      const void* grad_new_eff, const double* tdamp, double tstep, double e_trial, double e_est,
                      double branchcut, void* weights_inout, void* stream);

/* aiqmc_dmc_weights with the general arguments of comput_S as main_dmc.py drives it:
 *   e_trial_b / e_est_b (optional, device [B], ctx dtype): per-walker e_trial / e_est -- the
 *     driver's first block passes the per-walker pp energies of total_e (main_dmc.py:115-116);
 *     NULL: the scalars e_trial / e_est;
 *   cut_minima (optional, device double[2]): the e_cut minima for eloc_old / eloc_new
 *     (S_matrix.py:21-22: ONE jnp.min over the stacked arrays of ALL devices and the branch
 *     cut) -- a multi-GPU run all-reduces aiqmc_dmc_cut_minima with MIN and passes the result;
 *     NULL: computed from this batch. */
int aiqmc_dmc_weights_ex(aiqmc_ctx* ctx, int32_t B, const void* eloc_old, const void* eloc_new,
                         const void* grad_eff_old, const void* grad_new_eff, const double* tdamp, double tstep,
                         const void* e_trial_b, const void* e_est_b, double e_trial, double e_est, double branchcut,
                         const double* cut_minima, void* weights_inout, void* stream);

/* This batch's e_cut minima (S_matrix.py:21-22) for eloc_old / eloc_new: out (device
 * double[2]) = min(branchcut, min_b |e_est_b - eloc_b|) (e_est_b optional as above). */
int aiqmc_dmc_cut_minima(aiqmc_ctx* ctx, int32_t B, const void* eloc_old, const void* eloc_new, const void* e_est_b,
                         double e_est, double branchcut, double* out, void* stream);

/* Stochastic comb (DMC/branch.py:10-33) with the uniform draw u in [0,1):
 * newinds[B] (int32, device) = searchsorted(cumsum(w), (u wtot + j wtot/B) mod wtot),
 * weight_out[1] = wtot / B (device, ctx dtype). */
int aiqmc_dmc_branch(aiqmc_ctx* ctx, int32_t B, const void* weights, double u, int32_t* newinds, void* weight_out,
                     void* stream);

/* Pseudopotential tables (pphamiltonian.local_energy arguments,
 * Energy/pphamiltonian.py:130-146; shapes as the example drivers pass them,
 * example/single_atom_C/single_atom_C.py:13-23).  All HOST pointers; the
 * nonlocal arrays have list_l + 1 angular channels (P_l of
 * pseudopotential.py:250-269 returns list_l + 1 terms). */
typedef struct aiqmc_ecp {
  int32_t list_l;               /* 0..3                                       */
  int32_t n_local;              /* KL = Rn_local.shape[1]                     */
  int32_t n_nonlocal;           /* KN = Rn_non_local.shape[2]                 */
  const double* rn_local;       /* [A][KL]  (r**(n-2), pseudopotential.py:95) */
  const double* local_coes;     /* [A][KL]                                    */
  const double* local_exps;     /* [A][KL]                                    */
  const double* rn_non_local;   /* [A][list_l+1][KN]  (r**n, :150)            */
  const double* non_local_coes; /* [A][list_l+1][KN]                          */
  const double* non_local_exps; /* [A][list_l+1][KN]                          */
} aiqmc_ecp;

/* Attach pseudopotential tables to the context (replaces the closure
 * arguments of pphamiltonian.local_energy).  The potential charges of the
 * context (aiqmc_cfg.charges) are the effective core charges Z_eff. */
int aiqmc_set_ecp(aiqmc_ctx* ctx, const aiqmc_ecp* ecp);

/* Complex pseudopotential local energy of B walkers (the reference's
 * pphamiltonian.local_energy(...) -> _e_l(params, key, data), vmapped with one
 * key per walker, loss.py:203-204):
 *   e_re + i e_im = V_ee + V_nn + KE + local pp + nonlocal pp
 * with the nonlocal quadrature over the 50-point grid rotated by one random
 * orthogonal matrix per walker (pseudopotential.py:233-241).
 * rng_mode AIQMC_RNG_HOST: rot = device [B][3][3] (row-major, ctx dtype), the
 *   matrix jax.random.orthogonal would return; AIQMC_RNG_PHILOX: rot may be
 *   NULL, Haar O(3) matrices are drawn from (seed, offset).
 * logabs_q / phase_q (optional, [B][N][A][50]): log|psi| and phase at the
 * quadrature configurations, electron i moved to r_ia * (p_q R). */
int aiqmc_local_energy_ecp(aiqmc_ctx* ctx, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                           uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* logabs_q,
                           void* phase_q, void* stream);

/* The same with complex_output=True (pphamiltonian.local_energy(..., complex_output=True),
 * Energy/pphamiltonian.py:84-104, whose kinetic phase branch is hamiltonian.py:110-130): the
 * kinetic energy's phase terms + 1/2 |grad theta|^2 - i (lap theta / 2 + grad log|psi| . grad theta)
 * are added to e_re / e_im, theta = arg psi.  Two local-energy launch pairs (log|psi|, theta). */
int aiqmc_local_energy_ecp_complex(aiqmc_ctx* ctx, const void* pos, int32_t B, int32_t rng_mode, const void* rot,
                                   uint64_t seed, uint64_t offset, void* e_re, void* e_im, void* stream);

/* DMC T-moves (DMC/Tmoves.py:32-225, called per walker by dmc.py:79 before the
 * drift-diffusion step), in place on pos_inout [B][3N]: for every electron the
 * pp quadrature configurations of aiqmc_local_energy_ecp give the amplitudes
 * ratio * sum_l (exp(-tstep v_l) - 1) P_l(cos); one configuration per electron
 * is selected with the reference's cdf / searchsorted rule and accepted with
 * Re(norm / back_norm) > u (quirks T1-T8, oracle/dmc.py).  Needs aiqmc_set_ecp.
 * rng_mode AIQMC_RNG_HOST: rot [B][3][3] (get_rot's matrix), u_sel [B]
 *   (select_walker's uniform, one per walker, shared by its electrons) and
 *   u_acc [B][N] (the acceptance uniforms), device arrays of the ctx dtype;
 * AIQMC_RNG_PHILOX: all three drawn from (seed, offset).
 * acceptance (optional, [B][N], ctx dtype): Re(norm / back_norm). */
int aiqmc_dmc_tmoves(aiqmc_ctx* ctx, void* pos_inout, int32_t B, double tstep, int32_t rng_mode, const void* rot,
                     const void* u_sel, const void* u_acc, uint64_t seed, uint64_t offset, void* acceptance,
                     void* stream);

/* Energy statistics of one VMC iteration (constants.pmean_stats; the reference's two pmeans,
 * AIQMCrelease3 Loss/loss.py:206-208).  e_l[n] (dtype AIQMC_F32 | AIQMC_F64, device memory) is
 * reduced in fp64 into out[0..3] = [sum |e - m|^2, n m, n m^2, n] (m = the mean of these n
 * energies), one workgroup; the 4-vectors of all ranks sum (one all-reduce) to the pooled
 * statistics.  finalize != 0 also writes out[4..5] = [mean, variance] of these n energies.
 * aiqmc_energy_stats_final writes out[4..5] from a summed out[0..3].  out: >= 6 device doubles. */
int aiqmc_energy_stats(const void* e_l, int32_t dtype, int64_t n, double* out, int32_t finalize, void* stream);
int aiqmc_energy_stats_final(double* out, void* stream);

/* The energy-gradient weights of make_loss on ONE rank (Loss/loss.py:73-135 clipping with the
 * mean as centre, :206-208 statistics, :256-265 tangent weights), one launch: for local energies
 * e = e_re + i e_im (e_im NULL: real) of n walkers,
 *   stats[0..4] = [Re mean, Im mean, variance mean|e - mean|^2, Re centre, Im centre],
 *   w_re[b] = wscale Re(diff_b),  w_im[b] = wscale Im(diff_b + aux_b)  (w_im may be NULL),
 *   clipped_re/im[b] = aux.clipped_energy (may be NULL),
 * with clip_scale > 0: total-variation window around the mean per component, diff = clipped -
 * centre, centre = mean(clipped) (center_at_clipped) or the mean, aux = centre; clip_scale <= 0:
 * diff = e - mean, aux = e.  Sums in double, fixed order.  (Several ranks: the statistics need
 * all-reduces between the stages; the Python layer keeps its torch path there.) */
int aiqmc_loss_weights(const void* e_re, const void* e_im, int32_t dtype, int64_t n, double clip_scale,
                       int32_t center_at_clipped, double wscale, void* w_re, void* w_im, void* clipped_re,
                       void* clipped_im, double* stats, void* stream);

/* The same statistics, clipping and gradient weights over SEVERAL ranks, as three levels whose
 * rank partials sum with one all-reduce each (Loss/loss.py:107,206,208 and the gradient pmean of
 * Optimizer/adam.py:55).  aiqmc_loss_level(level, ...) for this rank's n energies:
 *   level 1: out[0..5] = L1 = [sum |e - m|^2, n Re m, n Im m, n |m|^2, n, #(Im e != 0)]  (m: rank mean)
 *   level 2: out[0..1] = L2 = [sum |Re e - Re E|, sum |Im e - Im E|]  from the SUMMED L1 (clipping only)
 *   level 3: from the summed L1 (and L2 when clip_scale > 0): the clipped energies xc (the total-
 *            variation window around the mean, clipped_re/im, may be NULL), the gradient weights
 *            w[0][b] = wscale (Re xc_b - Re E), w[1][b] = wscale (g0 != 0; centre at the clipped mean),
 *            wp[b] = the phase weight (wscale Im xc clipping, wscale (2 Im e - Im E) without; may be NULL),
 *            and out[0..1] = [sum Re xc, sum Im xc].
 * The caller then forms G = w[0]-weighted d log|psi| + wp-weighted d phase and G0 = w[1]-weighted
 * d log|psi| (aiqmc_param_grad_weighted), packs L3 = [out[0..1], G, G0] (aiqmc_loss_pack: double
 * L3[2 + 2P]), all-reduces it, and aiqmc_loss_final writes the pmean'd gradient
 * grad = (G - (Re dc - Re E) G0) / world (ctx dtype) and stats[0..5] = [Re E, Im E, variance,
 * Re dc, Im dc, #(Im e != 0) over all ranks] (dc: the clipped mean when center_at_clipped, else E).
 * L1/L2/L3/out/stats are device doubles; weights and energies of `dtype`. */
int aiqmc_loss_level(int32_t level, const void* e_re, const void* e_im, int32_t dtype, int64_t n,
                     const double* L1, const double* L2, double clip_scale, double wscale, int32_t g0, void* w,
                     void* wp, void* clipped_re, void* clipped_im, double* out, void* stream);
int aiqmc_loss_pack(const void* g, const void* gp, const void* g0, int32_t dtype, int32_t P, double* L3,
                    void* stream);
int aiqmc_loss_final(const double* L1, const double* L3, int32_t P, int32_t g0, int32_t center_at_clipped,
                     int32_t world, int32_t dtype, void* grad, double* stats, void* stream);

/* Optional HIP-event timing of the hot kernels, recorded on the caller's
 * stream around each launch while enabled.  Slots: 0 = proposal
 * value+gradient launches of aiqmc_mc_step, 1 = walker gradient launches of
 * aiqmc_mc_step, 2 = aiqmc_local_energy launches, 3 = value-only launches of
 * the ECP quadrature configurations.  aiqmc_profile_read waits
 * for the recorded events, returns the summed kernel time in ms and the launch
 * count of one slot, and clears it. */
int aiqmc_profile_enable(aiqmc_ctx* ctx, int32_t on);
int aiqmc_profile_read(aiqmc_ctx* ctx, int32_t slot, double* total_ms, int64_t* launches);

/* Diagnostics: aiqmc_logpsi_grad through the forward-mode kernel (the
 * production gradient is reverse mode); used to cross-check the two
 * derivative implementations at full batch size. */
int aiqmc_debug_logpsi_grad_forward(aiqmc_ctx* ctx, const void* pos, int32_t B, void* logabs, void* grad,
                                    void* stream);

/* Diagnostics: aiqmc_local_energy through the single-launch forward-Laplacian
 * kernel (second-order jets carried through the whole network).  The production
 * path (adjoint pass + first-derivative pass) must agree with it to rounding. */
int aiqmc_debug_local_energy_forward(aiqmc_ctx* ctx, const void* pos, int32_t B, void* e_l, void* logabs,
                                     void* grad, void* stream);

/* Diagnostics: aiqmc_mc_step evaluates each single-electron proposal from the
 * walker's cached electron stage and pair sums, recomputing only the moved
 * electron and its 2(N-1) pairs (default, on = 1).  on = 0 recomputes every
 * proposal from scratch; both must agree to rounding. */
int aiqmc_debug_set_proposal_reuse(aiqmc_ctx* ctx, int32_t on);

/* Waves per walker of the local energy's first-derivative pass (k_walker_lap): 1, 2 or 4, or
 * 0 (default) = the fewest that give >= 2 waves per SIMD for the batch (small per-GPU batches
 * under strong scaling split each walker over more waves).  Results agree to rounding. */
int aiqmc_debug_set_lap_waves(aiqmc_ctx* ctx, int32_t waves);

/* Diagnostics: aiqmc_mc_step applies the acceptance of every sweep but the last inside the
 * next sweep's walker launch (default, on = 1); on = 0 runs a separate acceptance launch per
 * sweep.  Both are bitwise identical (same arithmetic, same order). */
int aiqmc_debug_set_fuse_accept(aiqmc_ctx* ctx, int32_t on);

/* Diagnostics: from the second sweep of an aiqmc_mc_step call on, the walker launch's
 * Gauss-Jordan elimination takes the walker's pivot order of the previous sweep (default,
 * reuse = 1; partial pivoting only when a pivot comes out below 0.1 of the previous one);
 * reuse = 0 runs partial pivoting in every sweep.  Results agree to rounding. */
int aiqmc_debug_set_walker_pivots(aiqmc_ctx* ctx, int32_t reuse);

/* Diagnostics (host only, no GPU call): dynamic LDS bytes per workgroup and waves per workgroup
 * of the launches of shape (N, A) that size their LDS at launch time -- the part of a kernel's
 * LDS that a profiler's dispatch record does not report.  kind: AIQMC_LDS_*; dtype AIQMC_F32 /
 * AIQMC_F64.  waves = 0: chosen per launch (the first-derivative pass: 1, 2 or 4 by batch size).
 * (profiles/summarize.py joins this with the code objects' register counts.) */
#define AIQMC_LDS_PROPOSAL 0   /* k_walker_rev, Metropolis proposals from the walker cache */
#define AIQMC_LDS_WALKER 1     /* k_walker_rev, walker launches / value + gradient */
#define AIQMC_LDS_ADJOINT 2    /* k_walker_rev<PREP>, local energy adjoint pass */
#define AIQMC_LDS_LAP 3        /* k_walker_lap, local energy first-derivative pass */
#define AIQMC_LDS_PGRAD 4      /* k_param_grad */
#define AIQMC_LDS_FWDLAP 5     /* k_walker<LAP>, forward-Laplacian diagnostics */
int aiqmc_debug_launch_lds(int32_t nelectrons, int32_t natoms, int32_t dtype, int32_t kind, int32_t* bytes,
                           int32_t* waves);

/* Diagnostics: walker launches of systems with N <= 8 electrons run several walkers per wave
 * (default, on = 1: four for N <= 4, two for N <= 8); on = 0 runs one wave per walker.
 * Results agree to rounding. */
int aiqmc_debug_set_packed_walkers(aiqmc_ctx* ctx, int32_t on);

/* Diagnostics: the ECP quadrature's value launch for N <= 8 (k_quad_value) factors each displaced
 * configuration's matrix in its walker's recorded pivot order and re-runs partial pivoting only for
 * a configuration whose pivot falls below 0.1 of the walker's; on = 1 takes partial pivoting for
 * every configuration (the fallback path everywhere).  Results agree to rounding. */
int aiqmc_debug_set_quad_pivoted(aiqmc_ctx* ctx, int32_t on);

/* Diagnostics: in fp32, aiqmc_mc_step can sum the two limdrift reductions of each sweep
 * (|grad|^2 over the walkers, over the proposals; VMCmcstep.py:11-14) inside the walker and
 * proposal launches, as exact 64-bit integer sums of |grad|^2 in units of 2^-16: no reduction
 * launches, and the same bits in any arrival order.  mode 1 (default) and 2 = always (mode 1
 * limited it to batches of at most 1,024 walkers before round 4), 0 = never: reduction launches that sum the same
 * integers in 32 workgroups (k_taueff_part; the same bits as the fused sums), 3 = never, with the
 * single-workgroup fp64 tree sum (k_taueff; fp64 always uses it; results agree with the integer
 * sums to the float rounding of v2). */
int aiqmc_debug_set_fuse_reduce(aiqmc_ctx* ctx, int32_t on);

/* Diagnostics: the fp32 limdrift factor (VMCmcstep.py:11-14) of n per-configuration |grad|^2
 * values (device floats `sumsq`) through one of the reductions aiqmc_mc_step uses: mode 0 = the
 * fused integer accumulators (tacc_add + taueff_wave), 1 = k_taueff_part + taueff_wave, 2 = the
 * fp64 tree sum (k_taueff).  Writes the factor to the HOST double *out (synchronises `stream`).
 * Non-finite values give NaN, as the reference's float sum does; huge ones a small factor. */
int aiqmc_debug_limdrift_factor(aiqmc_ctx* ctx, const void* sumsq, int32_t n, double tstep, int32_t mode,
                                double* out, void* stream);

/* Development builds (-DAQ_ABLATE) only: skip proposal-kernel phases (bit mask, walker_rev.h) to
 * time their marginal cost; results are meaningless.  No effect in product builds. */
int aiqmc_debug_set_ablate(aiqmc_ctx* ctx, int32_t mask);

/* Diagnostics: shader-clock cycles per phase of the reverse-mode kernel, summed
 * over waves since the last call ([0..15] walker, [16..31] proposal launches);
 * all zero unless the library was built with -DAQ_PHASE_PROF. */
int aiqmc_debug_phase_cycles(aiqmc_ctx* ctx, uint64_t* out32);

/* Bytes of device workspace the context holds (for memory planning). */
int64_t aiqmc_workspace_bytes(const aiqmc_ctx* ctx);

const char* aiqmc_last_error(void);

/* Compile-time list of supported (N, A) shapes, as "N:A,N:A,...". */
const char* aiqmc_supported_shapes(void);

#ifdef __cplusplus
}
#endif
#endif /* AIQMC_H_ */
