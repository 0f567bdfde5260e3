/*
 * ccmpc.h -- C ABI of libccmpc.so, the MI355X (gfx950) implementation of CC-MPC's
 * Monte-Carlo prediction + MVOE chance-constraint path (planner v8ideal).
 *
 * The reference is pure Python (HyeontaeSung/CC-MPC, snapshot 2025-10-31).  Each entry point
 * below replaces one stage of its hot path; the reference function it replaces is cited as
 * file:line, relative to /root/reference/collect/in_simulation/midlevel/ unless stated.
 * The host-side mirror of the reference interface (cc-mpc_amd/ccmpc) binds these with ctypes;
 * INTEGRATION.md shows the binding a maintainer of the reference would add.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer unless its comment says "host".
 *  - All buffers are caller-allocated; no entry point allocates, frees or synchronises, so every
 *    call can be captured into a hipGraph.  Work is enqueued on `stream` (a hipStream_t; NULL =
 *    the null stream).  Calls are reentrant per stream.
 *  - Return value: CCMPC_OK (0) or a negative CCMPC_ERR_* code for bad arguments / launch
 *    failures (ccmpc_last_error() gives the message, per host thread).  Numerical failures of a
 *    single record (singular covariance, no real tangent, ...) do not fail the call; they are
 *    reported in that record's `status` field with a CCMPC_REC_* code, mirroring where the
 *    reference raises.
 *
 * Particle store ("plane-major SoA")
 *  - positions[(2*t + c) * ld + i], c = 0 for x, 1 for y: plane 2t+c holds coordinate c at step
 *    t of every particle.  Consecutive particles are consecutive in memory, so one wavefront
 *    reads 64 particles of one plane as a single coalesced burst.
 *  - A *cell* is one (obstacle vehicle, latent mode) pair; it owns particles
 *    [cell_off[c], cell_off[c] + cell_cnt[c]) in every plane.  cell_off must be a multiple of 4
 *    and ld a multiple of 4 (16-byte aligned 4-particle vectors).
 *  - dtype CCMPC_F64: world-frame float64 (what predict_ideal writes, v8ideal/__init__.py:2667).
 *    dtype CCMPC_F32: float32 relative to a per-cell origin (what Trajectron++ writes before
 *    `+ minpos`, v8ideal/__init__.py:486); every reduction promotes to float64 first.
 */
#ifndef CCMPC_H
#define CCMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *ccmpc_stream_t; /* hipStream_t */

#define CCMPC_ABI_VERSION 2

/* call status */
#define CCMPC_OK 0
#define CCMPC_ERR_ARG -1
#define CCMPC_ERR_LAUNCH -2
#define CCMPC_ERR_WORKSPACE -3
#define CCMPC_ERR_UNSUPPORTED -4

/* per-record status (0 = ok) */
#define CCMPC_REC_SINGULAR -10   /* inv(cov_tau) or solve(Sigma1, Sigma2) singular (LinAlgError) */
#define CCMPC_REC_NO_TANGENT -11 /* n^T Sigma n <= 0: choose_closest_tangent returns None tuple */
#define CCMPC_REC_NONFINITE -12  /* slope m or a moment is inf/nan (ref_y == mean_y, N_k < 2) */
#define CCMPC_REC_NOT_PD -13     /* conditional covariance not PD (np.linalg.cholesky raises) */
#define CCMPC_REC_NOT_PSD -14    /* sqrtm of an indefinite covariance would be complex */

/* particle dtypes */
#define CCMPC_F64 0
#define CCMPC_F32 1

/* One Minkowski/MVOE half-space (one (cell, t, tau) pair), 128 bytes.
 * Constraint on the ego position x_t:  side=+1:  n . x_t >= d ;  side=-1:  n . x_t <= d
 * (v8ideal/__init__.py:926-939).  The reference's (A, b) = (-n, -d) or (n, d). */
typedef struct ccmpc_halfspace {
  double n0, n1;          /* normal [-m, 1]                                            */
  double d;               /* offset of the chosen slope-m tangent                      */
  double q00, q01, q11;   /* Q  = MVOE(cov_infer*chi_r, cov_mu*chi_p)   (:915)           */
  double r00, r01, r11;   /* QR = MVOE(Q, R^2 I)                        (:917-918)       */
  double beta1, beta2;    /* fixed-point solutions of the two MVOE calls               */
  double lower_bound;     /* compute_lower_bound(cov_infer, cov_mu, cov_t, eps) (:942)   */
  double mean0, mean1;    /* ellipsoid centre = particle mean at step t (:896)         */
  int32_t which;          /* 0: the "+" tangent, 1: the "-" tangent                    */
  int32_t side;           /* +1 (>=) or -1 (<=)                                        */
  int32_t status;         /* CCMPC_REC_* or 0                                          */
  int32_t t_tau;          /* (t << 16) | tau                                           */
} ccmpc_halfspace;

/* One GMM-affine half-space (one (cell, t)), 128 bytes (v8ideal/__init__.py:1476-1515).
 * side=+1:  n . x_t >= rhs = d + margin ;  side=-1:  n . x_t <= rhs = d - margin
 * (plus the caller's S_big_repeated[0, t] term, which is a QP variable, not data). */
typedef struct ccmpc_affine_rec {
  double n0, n1, d;
  double margin;          /* Gamma * || sqrtm(cov) [m, -1]^T ||_2                       */
  double rhs;
  double mean0, mean1;
  double c00, c01, c11;   /* particle covariance at step t (ddof = 1)                  */
  double s00, s01, s11;   /* sqrtm(cov)                                                */
  double m;               /* slope -(ref_x - mean_x) / (ref_y - mean_y)                 */
  int32_t which, side, status, t;
} ccmpc_affine_rec;

/* The fields of a record the QP reads, 32 bytes: what the multi-GPU exchange moves instead of
 * the 128-byte record (the one collective is a record all-gather; no reference
 * counterpart -- the reference solves one scene per process).  rhs = the halfspace record's d
 * or the affine record's rhs; t_tau = the source record's last field. */
typedef struct ccmpc_gather_rec {
  double n0, n1, rhs;
  int16_t side, status;
  int32_t t_tau;
} ccmpc_gather_rec;

/* Pack n_rec records of kind CCMPC_REC_KIND_HALFSPACE / _AFFINE into ccmpc_gather_rec
 * (device pointers; one launch, 128 B read + 32 B written per record). */
int ccmpc_compact_records(const void *rec, int rec_kind, int64_t n_rec, ccmpc_gather_rec *out,
                          ccmpc_stream_t stream);

int ccmpc_abi_version(void);
const char *ccmpc_last_error(void);
const char *ccmpc_status_string(int status);

/* Stream-ordered copy of `bytes` between host (pinned) and device buffers, direction inferred
 * from the pointers (hipMemcpyDefault).  Graph plumbing with no reference counterpart: a
 * captured planning step (ccmpc/step.py) carries its packed input upload and output download
 * as graph nodes, so one replay is the whole step. */
int ccmpc_copy_async(void *dst, const void *src, size_t bytes, ccmpc_stream_t stream);
/* The same copy as a device kernel reading / writing the pinned host buffer directly (a graph
 * kernel node rather than a memcpy node); bytes and both pointers 16-byte aligned. */
int ccmpc_copy_kernel_async(void *dst, const void *src, size_t bytes, ccmpc_stream_t stream);

/* Stream-ordered signal: *host_word (pinned) = *value (device), visible to the host only after
 * every write this stream made before it (a system-scope release).  A captured step's host side
 * polls the word rather than synchronising the stream. */
int ccmpc_signal_host(int64_t *host_word, const int64_t *value, ccmpc_stream_t stream);
/* ccmpc_copy_kernel_async (device -> pinned host) and ccmpc_signal_host in one single-workgroup
 * launch: *host_word = *value becomes visible only after the copied bytes. */
int ccmpc_copy_signal_async(void *dst, const void *src, size_t bytes, int64_t *host_word,
                            const int64_t *value, ccmpc_stream_t stream);

/* Graph capture of a planning step (ccmpc/step.py): begin / end a relaxed-mode capture on
 * `stream` (the library calls and event record / wait pairs issued in between become the
 * graph; end instantiates it into *out_exec), replay it on a stream, release it.  The graph
 * holds the buffer addresses it was captured with: keep them alive while it exists, and let
 * its last replay finish before destroying it or them. */
int ccmpc_graph_capture_begin(ccmpc_stream_t stream);
int ccmpc_graph_capture_end(ccmpc_stream_t stream, void **out_exec);
int ccmpc_graph_launch(void *exec, ccmpc_stream_t stream);
int ccmpc_graph_destroy(void *exec);

/* ---------------------------------------------------------------------------------------
 * Moment (Gram) reduction.  Replaces every np.mean / np.cov over particle clouds on the path:
 *   v8ideal/__init__.py:864-875 (t=0 stats), :896 + makeconstraint.py:41-70 predict_moments
 *   (each (t,tau) np.cov is a 4x4 block of out_cov), :1485-1493 (affine), :2584-2606
 *   save_moments (mean_p0p1[t] = out_mean[t], cov_p0p1[t] = diagonal 2x2 block,
 *   cross_cov[t][tau] = block (t, tau)).
 * out_mean[c][t][2] (origin added back for F32), out_cov[c][2T][2T] (ddof = 1, symmetric).
 * n_particles_bound >= sum(cell_cnt) sizes the grid, so counts may be produced on the device.
 * T <= 40.  ONE kernel launch: per-chunk partial Gram sums are combined in-launch through a
 * fixed fan-in-16 tree of arrival counters (the last arriver of each group combines it), so
 * the result is deterministic and uses no float atomics.
 *
 * Workspace contract (every *_workspace_bytes-sized workspace): its first
 * round_up(workspace_bytes / 32, 256) bytes hold the tree's arrival counters, the rest the
 * partial-Gram slabs.  Zero-fill a fresh workspace ONCE (hipMemset after allocating); every
 * call leaves the counters zero again.  One workspace may serve calls of ANY shape (moments,
 * cycles, ideal rollouts, any T / cell count) as long as every call passes the same
 * workspace_bytes (the whole buffer) and that is >= the call's *_workspace_bytes: the counter
 * region depends on workspace_bytes only, so no call's slabs overwrite another call's
 * counters.  Do not share one workspace between concurrent streams.
 * ------------------------------------------------------------------------------------- */
size_t ccmpc_moments_workspace_bytes(int64_t T, int64_t n_cells, int64_t n_particles_bound);
int ccmpc_moments(const void *positions, int dtype, int64_t ld, int64_t T,
                  const double *origin /* [n_cells][2] for F32, NULL for F64 */,
                  const int64_t *cell_off, const int64_t *cell_cnt, int64_t n_cells,
                  int64_t n_particles_bound, void *workspace, size_t workspace_bytes,
                  double *out_mean, double *out_cov, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Minkowski / MVOE half-space assembly for every (cell, t, tau < t), from ccmpc_moments output.
 * Replaces v8ideal/__init__.py:893-947 with makeconstraint.py predict_moments (:41-70),
 * compute_mvoe (:7-38, called twice), choose_closest_tangent (:176-207) and
 * compute_lower_bound (:282-303).
 *  ref_traj[r][t][2]   reference trajectory r (host load_refT, :2768-2787), cell c uses
 *                      r = cell_ref[c] (NULL -> 0)
 *  cell_risk[c][3]     {chi_r = chi2.ppf(1-eps_ijt, 2), chi_p = chi2.ppf(0.9999, 2),
 *                       gamma = norm.ppf(1-eps_ijt)}, eps_ijt = eps_ura[ov,k]/ph (:910-913)
 *  R                   3.4 (:795); tol 1e-8, maxiter 1000 (makeconstraint.py:7)
 *  out_rec[c][T(T-1)/2] in the reference's append order: pair p = t(t-1)/2 + tau
 *  out_prob_lower[c][T] min over tau of the lower bound, 1.0 at t = 0 (:898, :943)
 * ------------------------------------------------------------------------------------- */
int ccmpc_minkowski(const double *mean, const double *cov, int64_t T, int64_t n_cells,
                    const double *ref_traj, const int32_t *cell_ref, const double *cell_risk,
                    double R, double tol, int32_t maxiter, ccmpc_halfspace *out_rec,
                    double *out_prob_lower, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * One-launch Minkowski constraint-generation cycle: ccmpc_moments + ccmpc_minkowski fused.
 * The last-arriving workgroup of each cell finalises its moments and immediately assembles the
 * cell's T(T-1)/2 half-spaces, so one planning step's obstacle constraints cost one kernel
 * (v8ideal/__init__.py:881-947 and the save_moments statistics :2575-2606).
 * Same arguments and outputs as the two calls it replaces; same workspace contract.
 * ------------------------------------------------------------------------------------- */
int ccmpc_minkowski_cycle(const void *positions, int dtype, int64_t ld, int64_t T,
                          const double *origin, const int64_t *cell_off, const int64_t *cell_cnt,
                          int64_t n_cells, int64_t n_particles_bound, void *workspace,
                          size_t workspace_bytes, const double *ref_traj, const int32_t *cell_ref,
                          const double *cell_risk, double R, double tol, int32_t maxiter,
                          double *out_mean, double *out_cov, ccmpc_halfspace *out_rec,
                          double *out_prob_lower, ccmpc_stream_t stream);

/* The same call with its arguments in one struct, filled once by a caller that launches the
 * same cycle every step (the argument marshalling of a 22-argument foreign call is microseconds
 * of host time in front of every launch from an interpreter).  ccmpc_cycle_args_size() =
 * sizeof(ccmpc_cycle_args), for a binding to check its layout. */
typedef struct ccmpc_cycle_args {
  const void *positions;
  int32_t dtype, maxiter;
  int64_t ld, T;
  const double *origin;
  const int64_t *cell_off, *cell_cnt;
  int64_t n_cells, n_particles_bound;
  void *workspace;
  size_t workspace_bytes;
  const double *ref_traj;
  const int32_t *cell_ref;
  const double *cell_risk;
  double R, tol;
  double *out_mean, *out_cov;
  ccmpc_halfspace *out_rec;
  double *out_prob_lower;
  ccmpc_stream_t stream;
} ccmpc_cycle_args;
int ccmpc_minkowski_cycle_args(const ccmpc_cycle_args *args);
size_t ccmpc_cycle_args_size(void);

/* ---------------------------------------------------------------------------------------
 * GMM-affine half-spaces for every (cell, t).  Replaces v8ideal/__init__.py:1470-1515.
 *  cell_gamma[c] = norm.ppf(1 - eps_ura[ov,k]/ph) (:1481-1482); out_rec[c][T].
 * ------------------------------------------------------------------------------------- */
int ccmpc_affine(const double *mean, const double *cov, int64_t T, int64_t n_cells,
                 const double *ref_traj, const int32_t *cell_ref, const double *cell_gamma,
                 double R, ccmpc_affine_rec *out_rec, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * GMM-affine half-spaces with the recursive-feasibility covariance scale, for every (cell, t):
 * compute_obstacle_constraints_GMM_affine_scale_ideal (v8ideal/__init__.py:2320-2425), and with
 * scaled = 0 its unscaled twin compute_obstacle_constraints_GMM_affine_robust (:1541-1878).
 *  scale(t) = max(1, max_{tau<t} compute_scale(predict_moments(t, tau), Gamma, chi_p))
 *             (makeconstraint.py:259-280) if scaled, else 1; cov = scale C_tt
 *  cell_risk[c][3]     as ccmpc_minkowski_cycle (chi_p = chi2.ppf(0.9999, 2), Gamma = norm.ppf(1 - eps))
 *  tangent_in[c][T]    slope m per (cell, t); NULL -> m from ref_traj (the T == ph case)
 *  const_idx_in[c][T]  with tangent_in: CCMPC_TANGENT_CHOOSE (-2) = the reference's None (closest
 *                      tangent to ref), or -1 / 0 / 1 = the index it passes (Python indexing; -1 is
 *                      the last candidate and is also what the record reports in `which`)
 * Constraint: n.x >= rhs (side +1) or <= rhs (side -1), rhs = d +/- Gamma sqrt(|cov|_F) |[m, -1]|.
 * Record fields: c00/c01/c11 = the unscaled cov (what the generator saves), s00 = scale,
 * s01 = sqrt(|cov|_F) of the scaled cov, s11 = 0.
 * ------------------------------------------------------------------------------------- */
#define CCMPC_TANGENT_CHOOSE -2
int ccmpc_affine_scale(const double *mean, const double *cov, int64_t T, int64_t n_cells,
                       const double *ref_traj, const int32_t *cell_ref, const double *cell_risk,
                       double R, int32_t scaled, const double *tangent_in,
                       const int32_t *const_idx_in, ccmpc_affine_rec *out_rec,
                       ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * predict_ideal: affine conditional-Gaussian forward rollout (v8ideal/__init__.py:2620-2711)
 * from the PREVIOUS planning step's moments, which stay device-resident (no pickle round trip).
 *  prev_mean[s][T_src][2], prev_cov[s][2T_src][2T_src]  -- ccmpc_moments output of that step
 *  src_cell[c]         the reference's data_idx fallback, resolved by the host (:2650-2656)
 *  x0[c][2]            the shared initial draw (:2662-2665); NULL -> x0 = mean_0 + chol(cov_0) z,
 *                      z = Philox pair (0, 0, rng_cell[c], STREAM_IDEAL_X0)
 *  Z[c][t][2][n]       step noise (:2699-2700); NULL -> Philox pair (i, t, rng_cell[c], STREAM_IDEAL_Z)
 *  rng_cell[c]         RNG stream id per cell (NULL -> c), so results are identical however the
 *                      cells are sharded over GPUs
 *  out positions: cell c occupies [c*S, c*S + n_samples) of every plane, S = n_samples rounded
 *  up to a multiple of 4 (so the output is a valid ccmpc_moments store), dtype F64, slot t holds
 *  x_{t+1} (the reference's slot quirk).  T <= T_src - 1, ld >= n_cells * S.
 *  out_status[c]: 0 or CCMPC_REC_SINGULAR / CCMPC_REC_NOT_PD.
 * ------------------------------------------------------------------------------------- */
int ccmpc_ideal_rollout(const double *prev_mean, const double *prev_cov, int64_t T_src,
                        const int32_t *src_cell, int64_t n_cells, int64_t T, int64_t n_samples,
                        const double *x0, const double *Z, uint64_t seed,
                        const int32_t *rng_cell, double *out_positions, int64_t ld,
                        int32_t *out_status, ccmpc_stream_t stream);

/* Same rollout fused with the moment reduction: particles are generated in registers and
 * reduced without ever being written to HBM (the reference's only consumer of the 1e6-row
 * ideal trajectories is np.cov, :886-907 and :2586-2606).  Noise from Philox only.  Same
 * workspace contract as ccmpc_moments.  out_mean / out_cov as ccmpc_moments for T steps. */
size_t ccmpc_ideal_moments_workspace_bytes(int64_t T, int64_t n_cells, int64_t n_samples);
int ccmpc_ideal_moments(const double *prev_mean, const double *prev_cov, int64_t T_src,
                        const int32_t *src_cell, int64_t n_cells, int64_t T, int64_t n_samples,
                        const double *x0, uint64_t seed, const int32_t *rng_cell,
                        void *workspace, size_t workspace_bytes, double *out_mean,
                        double *out_cov, int32_t *out_status, ccmpc_stream_t stream);

/* The shrinking-horizon step (T < ph) in one launch: ideal rollout -> moments -> half-spaces
 * (v8ideal/__init__.py:824-825 + :881-947).  Arguments as ccmpc_ideal_moments plus the
 * ccmpc_minkowski ones. */
int ccmpc_ideal_minkowski_cycle(const double *prev_mean, const double *prev_cov, int64_t T_src,
                                const int32_t *src_cell, int64_t n_cells, int64_t T,
                                int64_t n_samples, const double *x0, uint64_t seed,
                                const int32_t *rng_cell, void *workspace, size_t workspace_bytes,
                                const double *ref_traj, const int32_t *cell_ref,
                                const double *cell_risk, double R, double tol, int32_t maxiter,
                                double *out_mean, double *out_cov, int32_t *out_status,
                                ccmpc_halfspace *out_rec, double *out_prob_lower,
                                ccmpc_stream_t stream);

/* As ccmpc_ideal_minkowski_cycle; seed_dev (nullable) points at the Philox seed in device
 * memory and overrides `seed`, so a captured graph draws a fresh rollout per replay (the
 * planning-step graphs of ccmpc/step.py write it with the step's packed inputs). */
int ccmpc_ideal_minkowski_cycle_ex(const double *prev_mean, const double *prev_cov,
                                   int64_t T_src, const int32_t *src_cell, int64_t n_cells,
                                   int64_t T, int64_t n_samples, const double *x0, uint64_t seed,
                                   const uint64_t *seed_dev, const int32_t *rng_cell,
                                   void *workspace, size_t workspace_bytes,
                                   const double *ref_traj, const int32_t *cell_ref,
                                   const double *cell_risk, double R, double tol, int32_t maxiter,
                                   double *out_mean, double *out_cov, int32_t *out_status,
                                   ccmpc_halfspace *out_rec, double *out_prob_lower,
                                   ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * GMM-latent particle sampler (Trajectron++ predict tail behind prediction.py:81-86):
 * z ~ Categorical(p(z|x)) by inverse CDF, per step a = mu + L eps (GMM2D.rsample, one
 * component, L = [[s0, 0], [s1 rho, s1 sqrt(1 - rho^2)]]), Unicycle integration (exact at
 * constant turn rate and acceleration; straight when |dphi| <= 1e-2), float32 as torch runs it.
 *  init_state[o][4]   x, y, heading, speed (scene-relative)
 *  latent_cdf[o][L]   cumulative p(z|x) (host), L <= 64
 *  gmm[o][L][T][5]    mu_dphi, mu_a, log sigma_dphi, log sigma_a, rho   (float32)
 *  out_z[o][N]        latent id per particle (the reference's argmax z, prediction.py:103)
 *  out_pos            F32 store in SAMPLE order: OV o occupies [o*S, o*S + N), S = round_up(N, 4)
 * Noise: z uses Philox (i, 0, g, STREAM_SAMPLER_Z), eps uses (i, t, g, STREAM_SAMPLER_EPS) with
 * g = ov_base + o the GLOBAL OV id, so a scene's draws do not depend on how scenes are sharded
 * over ranks or batched into calls.
 * PARITY UNPINNED upstream (absent submodule): checked against the repo's own restatement.
 * This is the synthetic mode (Philox z and eps, per-latent parameters); the upstream-shaped
 * boundary is ccmpc_sample_unicycle_ex below, of which this is the (PER_LATENT, NULL, NULL) case.
 * ------------------------------------------------------------------------------------- */
int ccmpc_sample_unicycle(const double *init_state, const double *latent_cdf, int64_t n_latent,
                          const float *gmm, int64_t n_ov, int64_t N, int64_t T, double dt,
                          uint64_t seed, int64_t ov_base, int32_t *out_z, float *out_pos,
                          int64_t ld, ccmpc_stream_t stream);

/* The sampler at the boundary Trajectron++ actually emits (prediction.py:81-86): torch draws
 * z (latent.sample_p, one-hot -> argmax as :103 does) and the decoder's noise eps (randn inside
 * GMM2D.rsample), and p_y_xz's GRU decoder is autoregressive, so every sample carries its OWN
 * GMM parameters per step.  Replaces the action draw + Unicycle.integrate_samples tail of
 * p_y_xz (:85) and the argmax of :103.
 *  gmm_layout CCMPC_GMM_PER_LATENT:   gmm[o][L][T][5] selected by z (as ccmpc_sample_unicycle)
 *             CCMPC_GMM_PER_PARTICLE: gmm[o][T][5][N] (particle-minor; needs z_in)
 *  z_in[o][N]       injected latent ids in [0, n_latent) (ids outside are clamped for memory
 *                   safety; the Python mirror rejects them), or NULL: Philox inverse CDF of
 *                   latent_cdf (which may be NULL when z_in is given)
 *  eps_in[o][T][2][N] injected standard-normal noise (float32), or NULL: Philox
 *  seed_dev         device copy of the Philox seed (read at launch, so a captured graph draws
 *                   fresh particles per replay), or NULL: `seed`
 * Per-step action a = mu + L eps with L = [[s0, 0], [s1 rho, s1 sqrt(clamp(1 - rho^2, 1e-5,
 * 1))]] (GMM2D's clamp), the L eps row summed before mu is added.  out_z / out_pos as above.
 * PARITY UNPINNED upstream (Trajectron++ absent): checked against the repo's restatement. */
#define CCMPC_GMM_PER_LATENT 0
#define CCMPC_GMM_PER_PARTICLE 1
int ccmpc_sample_unicycle_ex(const double *init_state, const double *latent_cdf, int64_t n_latent,
                             const float *gmm, int32_t gmm_layout, const int32_t *z_in,
                             const float *eps_in, int64_t n_ov, int64_t N, int64_t T, double dt,
                             uint64_t seed, const uint64_t *seed_dev, int64_t ov_base,
                             int32_t *out_z, float *out_pos, int64_t ld, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Particle bucketing by latent mode: make_ovehicles (v8ideal/__init__.py:469-505) +
 * OVehicle.from_trajectron (ovehicle.py:24-117) on the sampler's sample-order store.
 *  keep_map[o][L]   kept-mode index of each latent value, -1 if p(z|x) <= filter (host decides;
 *                   latent_probs are host data); n_kept[o] >= 1 (the reference cannot regroup
 *                   into zero modes); cell_base[o] = first global cell of OV o
 *  minpos[o][2]     scene origin added in float64 to the float32 predictions (:486)
 *  region[o]        first slot of OV o's region in pos_out (4-aligned; each region needs
 *                   N + 4 * n_kept[o] slots)
 *  out: pos_out     F32 store (origin = minpos), cells in (ov, kept mode) order, each cell's
 *                   particles in the reference's order (native mode in sample order, then the
 *                   regrouped rare modes in ascending latent order, each in sample order)
 *       cell_off/cell_cnt [n_cells], cell_pmf = N_k / N, init_center [n_cells][2] (world)
 * Rare particles go to the kept mode whose centre (mean final position) is nearest, first
 * index on ties (scipy.spatial.distance_matrix + np.argmin).  Deterministic.
 * Workspace: ccmpc_bucket_workspace_bytes; its head holds the per-OV and per-chunk (16 blocks
 * of 256 particles) arrival counters, so zero-fill it once (every call leaves them zero).
 * Three launches.
 * ------------------------------------------------------------------------------------- */
size_t ccmpc_bucket_workspace_bytes(int64_t n_ov, int64_t N, int64_t n_latent, int64_t max_k);
int ccmpc_bucket(const int32_t *z, const float *pos_in, int64_t ld_in, int64_t T, int64_t n_ov,
                 int64_t N, int64_t n_latent, const int32_t *keep_map, const int32_t *n_kept,
                 const int32_t *cell_base, int64_t max_k, const double *minpos,
                 const int64_t *region, void *workspace, size_t workspace_bytes, float *pos_out,
                 int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
                 double *init_center, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * The reference's own prediction boundary into ccmpc_bucket's input.  Replaces the per-OV
 * `predictions[idx]` / `z[idx]` reads of make_ovehicles (v8ideal/__init__.py:469-490) on the
 * 5-tuple generate_vehicle_latents returns (prediction.py:93-105):
 *  pred[row][N][T][2]  float32, scene-relative (numpy's swapaxes(predictions, 0, 1) layout)
 *  z[row][N]           latent ids, int64 (z_bytes = 8: np.argmax's dtype) or int32 (4).
 *                      make_ovehicles indexes a list of n_latent entries by them (:488-491):
 *                      an id in [-n_latent, 0) wraps as a Python index; any other id outside
 *                      [0, n_latent) is where the reference raises IndexError -- it is counted
 *                      into z_bad[o] (and clamped, for memory safety, so the output is then
 *                      not the reference's: the caller must refuse it)
 *  rows[n_ov]          device int32: the node row of OV o (make_ovehicles skips the ego's
 *                      node); NULL = rows 0 .. n_ov-1
 *  out: pos_out        F32 sample-order store, OV o at o * ov_stride (ov_stride >= N, 4-aligned
 *                      for ccmpc_bucket): pos_out[(2t + c) * ld_out + o * ov_stride + i]
 *       z_out[n_ov][N] int32, as ccmpc_bucket reads it
 *       z_bad[n_ov]    device int32, optional (NULL): invalid ids of OV o ADDED (the caller
 *                      zero-fills it first)
 * One launch; traffic 2 x 8 T B per particle.  The step graph uses the one-pass placement
 * ccmpc_bucket_predictions below instead (no sample-order store).
 * ------------------------------------------------------------------------------------- */
int ccmpc_load_predictions(const float *pred, const void *z, int z_bytes, const int32_t *rows,
                           int64_t n_ov, int64_t N, int64_t T, int64_t n_latent, float *pos_out,
                           int64_t ld_out, int64_t ov_stride, int32_t *z_out, int32_t *z_bad,
                           ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Sampler + bucketing as one placement pass, for clouds of N <= 262144 particles per OV: the
 * same draws as ccmpc_sample_unicycle_ex (same Philox streams, same float32 arithmetic)
 * bucketed as ccmpc_bucket buckets them -- every cell holds the same particles in the same
 * order and the same init_center / pmf bits.  Replaces prediction.py:81-86 +
 * v8ideal/__init__.py:469-505 + ovehicle.py:24-117.  Launches: latent ids + counts, then the
 * sampler writing each native particle straight into its cell (rare ones into a rare list),
 * then the rare particles' placement -- one launch up to N = 8192, keys then copy above it.
 * Differences from ccmpc_bucket's output: only where the cells start.  Cell k of OV o starts at
 *   region[o] + sum_{j<k} round4(n_j + R_o)   (n_j = mode j's own particles, R_o = rare ones)
 * so region[o] needs n_kept[o] * (N + 4) free slots of pos_out.  out_z (optional, may be NULL)
 * gets the sample-order latent ids.  N > 262144: the sampler + ccmpc_bucket.
 * Workspace: ccmpc_sample_bucket_workspace_bytes (0 = shape not supported), 256-byte aligned;
 * no initialisation needed (the first launch writes everything the second reads).
 * ------------------------------------------------------------------------------------- */
size_t ccmpc_sample_bucket_workspace_bytes(int64_t n_ov, int64_t N, int64_t T, int64_t max_k);
int ccmpc_sample_bucket(const double *init_state, const double *latent_cdf, int64_t n_latent,
                        const float *gmm, int32_t gmm_layout, const int32_t *z_in,
                        const float *eps_in, int64_t n_ov, int64_t N, int64_t T, double dt,
                        uint64_t seed, const uint64_t *seed_dev, int64_t ov_base,
                        const int32_t *keep_map, const int32_t *n_kept, const int32_t *cell_base,
                        int64_t max_k, const double *minpos, const int64_t *region,
                        void *workspace, size_t workspace_bytes, int32_t *out_z, float *pos_out,
                        int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
                        double *init_center, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * make_ovehicles (v8ideal/__init__.py:469-505, ovehicle.py:24-117) on the reference's own
 * predictor output in ONE placement pass: ccmpc_sample_bucket's launches with the predictor's
 * coordinates in place of the sampler (no sample-order store, no re-read + scatter of every
 * particle).  Inputs as ccmpc_load_predictions (pred[row][N][T][2] float32 scene-relative,
 * z[row][N] int64 / int32, rows[n_ov] or NULL); bucketing arguments and outputs as
 * ccmpc_sample_bucket (its workspace size: ccmpc_sample_bucket_workspace_bytes(n_ov, N, T,
 * max_k)); cells bit-identical to ccmpc_load_predictions + ccmpc_bucket.
 *  z_bad[n_ov]  device int32, optional: the number of OV o's ids make_ovehicles' list index
 *               would refuse (outside [-n_latent, n_latent); [-n_latent, 0) wraps) -- WRITTEN
 *               (no zero-fill needed).  Non-zero: the reference raises IndexError there, and
 *               the output is not the reference's (those ids were clamped).
 * ------------------------------------------------------------------------------------- */
int ccmpc_bucket_predictions(const float *pred, const void *z, int z_bytes, const int32_t *rows,
                             int64_t n_ov, int64_t N, int64_t T, int64_t n_latent,
                             const int32_t *keep_map, const int32_t *n_kept,
                             const int32_t *cell_base, int64_t max_k, const double *minpos,
                             const int64_t *region, void *workspace, size_t workspace_bytes,
                             float *pos_out, int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,
                             double *cell_pmf, double *init_center, int32_t *z_bad,
                             ccmpc_stream_t stream);
/* The same with the predictor's tensors named at RUN time: ptrs (device memory, e.g. a field of
 * a captured graph's input pack) holds the addresses {pred, z} of that launch's tensors, so a
 * graph captured once reads each frame's predictor output in place (no device-to-device copy
 * into buffers of its own).  The tensors must stay alive until the launch's outputs are read. */
int ccmpc_bucket_predictions_indirect(const uint64_t *ptrs, int z_bytes, const int32_t *rows,
                                      int64_t n_ov, int64_t N, int64_t T, int64_t n_latent,
                                      const int32_t *keep_map, const int32_t *n_kept,
                                      const int32_t *cell_base, int64_t max_k,
                                      const double *minpos, const int64_t *region,
                                      void *workspace, size_t workspace_bytes, float *pos_out,
                                      int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,
                                      double *cell_pmf, double *init_center, int32_t *z_bad,
                                      ccmpc_stream_t stream);

/* The three placement calls above with the caller's input pack copied in the same first launch
 * (the planning-step graph's packed H2D copy): equal to
 *   ccmpc_copy_kernel_async(pack_dev, pack_host, pack_bytes, stream)
 * followed by the unpacked call, whose pointer arguments may point into pack_dev.  The latent-id
 * pass reads its own inputs (latent CDF, keep map, seed, z or the predictor's addresses) from the
 * pinned host side while the copy runs, so the copy's kernel boundary leaves the step.
 * pack_host: pinned host memory (device-accessible by its host address); pack_bytes % 16 == 0,
 * both pointers 16-byte aligned. */
int ccmpc_sample_bucket_packed(void *pack_dev, const void *pack_host, size_t pack_bytes,
                               const double *init_state, const double *latent_cdf,
                               int64_t n_latent, const float *gmm, int32_t gmm_layout,
                               const int32_t *z_in, const float *eps_in, int64_t n_ov, int64_t N,
                               int64_t T, double dt, uint64_t seed, const uint64_t *seed_dev,
                               int64_t ov_base, const int32_t *keep_map, const int32_t *n_kept,
                               const int32_t *cell_base, int64_t max_k, const double *minpos,
                               const int64_t *region, void *workspace, size_t workspace_bytes,
                               int32_t *out_z, float *pos_out, int64_t ld_out, int64_t *cell_off,
                               int64_t *cell_cnt, double *cell_pmf, double *init_center,
                               ccmpc_stream_t stream);
int ccmpc_bucket_predictions_packed(void *pack_dev, const void *pack_host, size_t pack_bytes,
                                    const float *pred, const void *z, int z_bytes,
                                    const int32_t *rows, int64_t n_ov, int64_t N, int64_t T,
                                    int64_t n_latent, const int32_t *keep_map,
                                    const int32_t *n_kept, const int32_t *cell_base,
                                    int64_t max_k, const double *minpos, const int64_t *region,
                                    void *workspace, size_t workspace_bytes, float *pos_out,
                                    int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,
                                    double *cell_pmf, double *init_center, int32_t *z_bad,
                                    ccmpc_stream_t stream);
int ccmpc_bucket_predictions_indirect_packed(void *pack_dev, const void *pack_host,
                                             size_t pack_bytes, const uint64_t *ptrs,
                                             int z_bytes, const int32_t *rows, int64_t n_ov,
                                             int64_t N, int64_t T, int64_t n_latent,
                                             const int32_t *keep_map, const int32_t *n_kept,
                                             const int32_t *cell_base, int64_t max_k,
                                             const double *minpos, const int64_t *region,
                                             void *workspace, size_t workspace_bytes,
                                             float *pos_out, int64_t ld_out, int64_t *cell_off,
                                             int64_t *cell_cnt, double *cell_pmf,
                                             double *init_center, int32_t *z_bad,
                                             ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Headings, bounding-box vertices and L4 outer approximation for every (cell, t).
 * Replaces ovehicle.py:72-76 (yaws = atan2 of step deltas, step 0 from past[-1]),
 * v8ideal/__init__.py:627-640 (vertices_of_bboxes, restated from midlevel/util.py:104-124),
 * :694-736 -> midlevel/util.py:171-200 (A = [I; -I] R(mean yaw), b = max_{particles, corners} A v)
 * and the t = 0 yaw statistics of :872, :875.
 *  past_last[c][2]   world-frame past[-1] of the cell's OV;  bbox[c][2] = {lon, lat}
 *  out_A[c][T][4][2], out_b[c][T][4], out_yaw_mean[c][T], out_yaw0_var[c] (ddof = 1)
 *  out_yaw (nullable)       pred_yaws in store layout [T][ld]
 *  out_vertices (nullable)  corners in store layout [T][8][ld], plane 8t + 2 corner + xy
 * ------------------------------------------------------------------------------------- */
int ccmpc_l4(const void *positions, int dtype, int64_t ld, int64_t T, const double *origin,
             const int64_t *cell_off, const int64_t *cell_cnt, int64_t n_cells,
             const double *past_last, const double *bbox, double *out_A, double *out_b,
             double *out_yaw_mean, double *out_yaw0_var, double *out_yaw, double *out_vertices,
             ccmpc_stream_t stream);

/* The same outputs with every (cell, t) split over ~n_particles_bound / (n_cells 1024) workgroups
 * in two launches (pass 1: headings and their sums; pass 2: corners and maxima; each
 * (cell, t)'s last arriving workgroup combines the chunks, sums in chunk order, so the result is
 * deterministic).  One workgroup per (cell, t) is issue-bound on its f64 atan2 / division work
 * for large clouds; this form spreads it over the chip.  Workspace: ccmpc_l4_workspace_bytes,
 * 256-byte aligned, its head (arrival counters) zero-filled once; every call leaves it zero. */
size_t ccmpc_l4_workspace_bytes(int64_t T, int64_t n_cells, int64_t n_particles_bound);
int ccmpc_l4_split(const void *positions, int dtype, int64_t ld, int64_t T, const double *origin,
                   const int64_t *cell_off, const int64_t *cell_cnt, int64_t n_cells,
                   int64_t n_particles_bound, const double *past_last, const double *bbox,
                   void *workspace, size_t workspace_bytes, double *out_A, double *out_b,
                   double *out_yaw_mean, double *out_yaw0_var, double *out_yaw,
                   double *out_vertices, ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * The caller of the path: the planning step's quadratic program,
 * batched over scenes.  Replaces the cvxpy + CPLEX problem of do_highlevel_control
 * (v8ideal/__init__.py:2850-2930, :2999-3012, :3040-3110) with the road-boundary MILP off (the reference
 * default, :217), so the problem is a convex QP in the controls u (2T values):
 *   state      x = Gamma_f (u - u_bar) + x_bar + Gamma_p u_prev            (:2877-2891)
 *   bounds     [min_a, -max_delta] <= (u[2t], u[2t+1]) <= [max_a, max_delta]  (:2874-2878)
 *              0 <= v_t <= max_v                                           (:610-626)
 *   obstacles  every record with status 0:  n . x_t >= d (side +1) or <= d (side -1)
 *              (Minkowski :926-939; affine: rhs, :1503-1515 with S_big = 0)
 *   objective  w_final |X_{T-1} - goal|^2 + sum_t w_ref |X_t - ref_t|^2
 *              + sum_t U_t^T R1 U_t + sum_{t>=1} dU_t^T R2 dU_t                (:2478-2507)
 * U = cp.reshape(u, (T, 2)) in the objective uses cvxpy's default column-major order
 * (U_t = (u[t], u[T+t]), CCMPC_U_ORDER_F) in the reference, while the bounds and Gamma's columns
 * interleave (accel, steer) per step; CCMPC_U_ORDER_C pairs the objective the same way.
 * Solved by a primal-dual interior point method (Mehrotra predictor-corrector), one workgroup
 * per scene, the whole iteration in LDS, then polished: the equality-constrained QP on the
 * IPM's active set, kept only when it is a verified KKT point (T <= 32; beyond, the IPM's
 * answer at tol).
 * ------------------------------------------------------------------------------------- */
#define CCMPC_U_ORDER_F 0
#define CCMPC_U_ORDER_C 1
#define CCMPC_REC_KIND_HALFSPACE 0 /* ccmpc_halfspace records [cells][T(T-1)/2] */
#define CCMPC_REC_KIND_AFFINE 1    /* ccmpc_affine_rec records [cells][T] */
/* the same records packed as ccmpc_gather_rec (ccmpc_compact_records): what the multi-GPU
 * record exchange moves, and what the QP can read in place after it */
#define CCMPC_REC_KIND_HALFSPACE_COMPACT 2
#define CCMPC_REC_KIND_AFFINE_COMPACT 3

/* QP status per scene */
#define CCMPC_QP_OK 0
#define CCMPC_QP_MAXITER 1      /* no verified solution within max_iter: infeasible (the
                                   reference returns InSimulationException, :3099-3110)   */
#define CCMPC_QP_NUMERIC 2      /* the objective's Hessian is not positive definite       */
#define CCMPC_QP_SKIPPED_ROWS 4 /* flag: records with status != 0 were left out */

/* QP method (environment CCMPC_QP_METHOD = "gi" / "ipm", read per ccmpc_mpc_qp call):
 * the Goldfarb-Idnani dual active-set method for n = 2T <= 16 (one wave per scene), the
 * Mehrotra interior point + active-set polish otherwise (and where the active-set solve
 * exceeds its step budget).  Both return the problem's unique minimiser (strictly convex). */
#define CCMPC_QP_METHOD_IPM 0
#define CCMPC_QP_METHOD_GI 1

typedef struct ccmpc_mpc_params {
  double w_final, w_ref;                     /* objective weights (:93-102)          */
  double w_accel, w_joint, w_turning;        /* R1                                   */
  double w_ch_accel, w_ch_joint, w_ch_turning; /* R2                                 */
  double min_a, max_a, max_delta, max_v;     /* control / speed limits (:88-109)     */
} ccmpc_mpc_params;

/* LTV model of the ego vehicle about u_init = 0, the only linearisation input the planner
 * uses (make_local_params, v8ideal/__init__.py:537-557 -> dynamics/bicycle_v2.py
 * VehicleModel.get_optimization_ltv :261-308).  Per scene:
 *  x_init[s][4] = [x, y, psi, v];  out_xbar[s][4T] = X_bar[1:];  out_gamma[s][4T][2T]. */
int ccmpc_mpc_ltv(const double *x_init, int64_t n_scenes, int64_t T, double Ts, double l_r,
                  double L, double *out_xbar, double *out_gamma, ccmpc_stream_t stream);

/* Workspace for scenes holding at most max_cells_per_scene cells of records. */
size_t ccmpc_mpc_qp_workspace_bytes(int64_t n_scenes, int64_t T, int64_t max_cells_per_scene,
                                    int rec_kind);

/* One QP per scene s, horizon T <= T_full, T_prev = T_full - T steps already executed:
 *  gamma[s][4 T_full][2 T_full], xbar[s][4 T_full]  (the full-horizon model of the first step)
 *  ubar[s][2 T_full] or NULL (= 0, u_init = 0);  u_prev[s][2 T_prev] or NULL when T_prev = 0
 *  goal[s][2];  ref[s][n_ref][2] (step t uses ref[min(t, n_ref - 1)], :2492-2501)
 *  rec: records of every scene's cells, scene s owning cells [scene_cell[s], scene_cell[s+1]),
 *       128-byte records (rec_kind CCMPC_REC_KIND_HALFSPACE / _AFFINE) or their 32-byte
 *       ccmpc_gather_rec packing (_HALFSPACE_COMPACT / _AFFINE_COMPACT): the same solve
 *  params: HOST pointer.
 *  out_u[s][2T] (the cvxpy variable u), out_x[s][T][4], out_cost[s], out_status[s],
 *  out_iter[s] (IPM iterations). */
int ccmpc_mpc_qp(int64_t n_scenes, int64_t T, int64_t T_full, const double *gamma,
                 const double *xbar, const double *ubar, const double *u_prev,
                 const double *goal, const double *ref, int64_t n_ref, const void *rec,
                 int rec_kind, const int64_t *scene_cell, int64_t max_cells_per_scene,
                 const ccmpc_mpc_params *params, int u_order, int32_t max_iter, double tol,
                 void *workspace, size_t workspace_bytes, double *out_u, double *out_x,
                 double *out_cost, int32_t *out_status, int32_t *out_iter,
                 ccmpc_stream_t stream);

/* ccmpc_mpc_qp with the LTV rebuild fused in (the planning frame at Tsh == ph: one launch
 * instead of ccmpc_mpc_ltv then ccmpc_mpc_qp).  Each scene's model about u = 0 is computed from
 * ltv->x_init[s][4] with ccmpc_mpc_ltv's arithmetic (the same bits), written to gamma / xbar
 * (OUTPUTS here, [s][4 T_full][2 T_full] and [s][4 T_full]: later frames pass them to
 * ccmpc_mpc_qp) and used by the solve without reading them back. */
typedef struct ccmpc_qp_ltv {
  const double *x_init; /* device, [n_scenes][4] */
  double Ts, l_r, L;
} ccmpc_qp_ltv;
int ccmpc_mpc_qp_ltv(const ccmpc_qp_ltv *ltv, int64_t n_scenes, int64_t T, int64_t T_full,
                     double *gamma, double *xbar, const double *u_prev, const double *goal,
                     const double *ref, int64_t n_ref, const void *rec, int rec_kind,
                     const int64_t *scene_cell, int64_t max_cells_per_scene,
                     const ccmpc_mpc_params *params, int u_order, int32_t max_iter, double tol,
                     void *workspace, size_t workspace_bytes, double *out_u, double *out_x,
                     double *out_cost, int32_t *out_status, int32_t *out_iter,
                     ccmpc_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * TEST ONLY (not a reference interface): the half-space tail's device functions -- the ones
 * ccmpc_minkowski_cycle / ccmpc_minkowski / ccmpc_affine_scale run per record -- on n batched
 * inputs, so the reference's component golden vectors reach the device arithmetic.  Device
 * pointers, float64, row-major 2x2 matrices (a, b, c, d):
 *  MVOE     in[n][8]  = S1, S2                 out[n][6]  = beta, Q, ok (1/0)
 *           (compute_mvoe, makeconstraint.py:7-38; tol / maxiter as the cycle's)
 *  TANGENT  in[n][10] = mu[2], Sigma, c, m, a[2]  out[n][5] = n[2], d, which, status (0 or
 *           CCMPC_REC_NO_TANGENT)  (choose_closest_tangent, makeconstraint.py:134-207)
 *  BOUND    in[n][14] = cov_infer, cov_mu, cov_t, Gamma, chi_p   out[n][2] = lower bound,
 *           scale  (compute_lower_bound / compute_scale, makeconstraint.py:259-303)
 *  PAIR     in[n][18] = 4x4 cov of (x_tau, y_tau, x_t, y_t), Gamma, chi_p
 *           out[n][14] = cov_infer, cov_mu, cov_t, lower bound, scale
 *           (predict_moments, makeconstraint.py:41-70, then BOUND)
 * ------------------------------------------------------------------------------------- */
#define CCMPC_SELFTEST_MVOE 0
#define CCMPC_SELFTEST_TANGENT 1
#define CCMPC_SELFTEST_BOUND 2
#define CCMPC_SELFTEST_PAIR 3
int ccmpc_selftest(int kind, int64_t n, const double *in, double *out, double tol,
                   int32_t maxiter, ccmpc_stream_t stream);

/* Test aid: fill every CU's LDS with `value` (tests/test_gpu_lds_poison.py runs the kernels
 * after NaN and after zero fills and requires the same bits: no kernel reads LDS it did not
 * write). */
int ccmpc_poison_lds(double value, ccmpc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CCMPC_H */
