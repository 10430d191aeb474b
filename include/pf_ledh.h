/*
 * pf_ledh.h — C ABI of the MI355X LEDH particle-flow filter (libpf_hip.so).
 *
 * Replaces the per-particle flow loop of the reference's LEDHFlowPF
 * (/root/reference/models/LEDH_particle_filter.py, cited "ledh.py:LINE"):
 * the Python mirror particle_filters_amd/ledh.py binds these entries with
 * ctypes exactly like pf_engine.h's.  Conventions (status codes, ownership,
 * one handle = one device + one stream, not re-entrant) are those of pf_engine.h.
 *
 * Arithmetic is fp64 (the reference's).  The Gaussian tracker (EKF/UKF,
 * ledh.py:13-16) never sees the particles, so the caller hands the engine its
 * predicted covariance P_k per step (pf_ledh_step) or the whole sequence P_1..P_T
 * up front (pf_ledh_run) — or lets the engine run the EKF itself on the device
 * (pf_ledh_run_ekf, pf_ledh_ekf_sequence).
 */
#ifndef PF_LEDH_H
#define PF_LEDH_H

#include <stdint.h>

#include "pf_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* process noise v of eta_0 = g(x, u) + v (ledh.py:108-115) */
#define PF_NOISE_NONE 0   /* v = 0: the reference default when process_noise_sampler is None */
#define PF_NOISE_HOST 1   /* caller-supplied v [N][nx] (a process_noise_sampler's draw) */
#define PF_NOISE_DEVICE 2 /* Philox normals times chol(Q) on the device */

/* flow evaluation */
#define PF_LEDH_FLOW_AUTO 0         /* shared-Jacobian path when h is linear (identical A^i, S^i for all
                                       particles), per-particle path otherwise */
#define PF_LEDH_FLOW_PER_PARTICLE 1 /* always linearise at every particle (ledh.py:140-179) */

typedef struct pf_ledh_opts {
  int64_t n_particles;       /* LEDHConfig.n_particles (ledh.py:46) */
  int32_t n_lambda;          /* LEDHConfig.n_lambda_steps (ledh.py:47), clamped to >= 1 (ledh.py:132) */
  double resample_ess_ratio; /* LEDHConfig.resample_ess_ratio (ledh.py:48); 0 disables resampling */
  uint64_t seed;             /* Philox key for PF_NOISE_DEVICE / device init / device resampling */
  int32_t device;
  int32_t flow_mode;         /* PF_LEDH_FLOW_* */
} pf_ledh_opts;

typedef struct pf_ledh_info {
  double ess;       /* effective_sample_size(w) of the normalised flow weights (ledh.py:39-41, 202) */
  int32_t resample; /* 1 if ess < ratio * N (ledh.py:201-203); applied by pf_ledh_resample */
  int32_t _pad;
} pf_ledh_info;

typedef struct pf_ledh_handle pf_ledh_handle;

/* LEDHFlowPF.__init__ (ledh.py:63-81).  model: g = trans_kind (+ additive noise v), h = obs_kind
 * with its analytic Jacobian; Q = covariance of the Gaussian transition density log_trans_pdf,
 * R = the measurement covariance (log_like_pdf and the flow's S^i, ledh.py:149). */
pf_status pf_ledh_create(const pf_model_desc* model, const pf_ledh_opts* opts, pf_ledh_handle** out);
void pf_ledh_destroy(pf_ledh_handle* h);
int32_t pf_ledh_model_supported(int32_t nx, int32_t nz, int32_t trans_kind, int32_t obs_kind);

/* init_from_gaussian (ledh.py:84-91): particles = mean0 + eps, uniform weights.
 * eps [N][nx] (the caller's rng.multivariate_normal draw) or NULL (device Philox times chol(cov0)).
 * mean_out [nx], cov_out [nx][nx] (nullable): _weighted_stats of the initial set. */
pf_status pf_ledh_init(pf_ledh_handle* h, const double* mean0, const double* cov0, const double* eps,
                       double* mean_out, double* cov_out);

/* One flow step up to the weights (ledh.py:104-195): P [nx][nx] = the tracker's predicted covariance
 * (symmetrised here, ledh.py:106), z [nz], u [nx] or NULL, noise PF_NOISE_* with v [N][nx] for
 * PF_NOISE_HOST.  info (nullable) gets the ESS and the resample decision; cond_S (nullable, [L][nz][nz])
 * gets S^0(lambda_j) of particle 0 for the reference's condition-number diagnostics (ledh.py:151-157). */
pf_status pf_ledh_step(pf_ledh_handle* h, const double* P, const double* z, const double* u, int32_t noise,
                       const double* v, pf_ledh_info* info, double* cond_S);

/* Apply the decided resample (ledh.py:201-206): U = the caller's uniform (rng.random()) or NULL
 * (device Philox).  Then (and also without a resample) the posterior mean/cov (ledh.py:209)
 * of the current state: mean [nx], cov [nx][nx] (nullable). */
pf_status pf_ledh_finish(pf_ledh_handle* h, const double* U, double* mean, double* cov);

/* State readout / injection.  particles [N][nx]; weights [N] (normalised). */
pf_status pf_ledh_get_particles(pf_ledh_handle* h, double* particles);
pf_status pf_ledh_get_weights(pf_ledh_handle* h, double* weights);
pf_status pf_ledh_set_state(pf_ledh_handle* h, const double* particles, const double* weights);

/* The whole T loop on the device with no host synchronisation inside T:
 * Ps [T][nx][nx] tracker covariances, Z [T][nz], U [T][nx] or NULL.  Noise PF_NOISE_NONE,
 * PF_NOISE_DEVICE (resampling uniforms from Philox) or PF_NOISE_HOST (the draws set by
 * pf_ledh_set_run_replay for a run of this T).  Outputs (host, nullable): means [T][nx],
 * covs [T][nx][nx], ess [T], flags [T].  A failed launch or grid-barrier timeout inside the run
 * leaves the handle uninitialised (PF_E_NOT_INITIALIZED on the next call): its state would be
 * part-advanced. */
pf_status pf_ledh_run(pf_ledh_handle* h, const double* Ps, const double* Z, const double* U, int64_t T,
                      int32_t noise, double* means, double* covs, double* ess, uint8_t* flags);

/* Replayed draws for the NEXT run of T steps (pf_ledh_run / pf_edh_run / pf_ledh_run_ekf with
 * noise PF_NOISE_HOST): step t's process noise v_t [N][nx] (the process_noise_sampler draw,
 * ledh.py:109-116) and its resampling uniform U_t (the rng.random() of systematic_resample,
 * ledh.py:28; read only when step t resamples).  The reference's generator consumes U_t only on
 * resampling steps, so a caller replaying its stream lays the draws out with the decisions it
 * expects (and checks the run's flags against them).  noise [T][N][nx], uniforms [T]; copied. */
pf_status pf_ledh_set_run_replay(pf_ledh_handle* h, const double* noise, const double* uniforms, int64_t T);

/* The Gaussian tracker on the device: the additive-noise EKF of extended_kalman_filter.py:164-241
 * (predict x = g(x), P = G P G^T + Qt; update with S = H P H^T + Rt, K = P H^T S^-1, P = (I - K H) P)
 * with the compiled model's analytic Jacobians, run over Z [T][nz] from (x0 [nx], P0 [nx][nx]).
 * Ps [T][nx][nx] (host, nullable) gets the symmetrised predicted covariances the flow uses
 * (ledh.py:105-106); x_final / P_final (nullable) the tracker's last posterior. */
pf_status pf_ledh_ekf_sequence(pf_ledh_handle* h, const double* x0, const double* P0, const double* Qt,
                               const double* Rt, const double* Z, int64_t T, double* Ps, double* x_final,
                               double* P_final);

/* pf_ledh_run with the device EKF as the tracker (no host work inside the run). */
pf_status pf_ledh_run_ekf(pf_ledh_handle* h, const double* x0, const double* P0, const double* Qt, const double* Rt,
                          const double* Z, const double* U, int64_t T, int32_t noise, double* means, double* covs,
                          double* ess, uint8_t* flags, double* x_final, double* P_final);

/* Measurement hooks: the handle's stream, synchronisation, and whether the last step used the
 * shared-Jacobian path. */
void* pf_ledh_stream(pf_ledh_handle* h);
pf_status pf_ledh_synchronize(pf_ledh_handle* h);
int32_t pf_ledh_shared_path(pf_ledh_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* PF_LEDH_H */
