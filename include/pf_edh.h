/*
 * pf_edh.h — C ABI of the MI355X EDH (exact Daum-Huang) particle-flow filter (libpf_hip.so).
 *
 * Replaces the per-particle flow loop of the reference's EDHFlowPF
 * (/root/reference/models/EDH_particle_filter.py, cited "edh.py:LINE"): EDHConfig 58-64,
 * init_from_gaussian 173-180, step 182-317.  The Python mirror particle_filters_amd/edh.py
 * binds these entries with ctypes.
 *
 * An EDH handle IS a pf_ledh_handle: pf_ledh_init (init_from_gaussian), pf_ledh_finish
 * (resample + _weighted_stats), pf_ledh_get_particles / get_weights / set_state,
 * pf_ledh_run_ekf (device EKF tracker), pf_ledh_stream / synchronize and pf_ledh_destroy
 * accept it unchanged.  Only the flow differs, and it needs one more tracker quantity than
 * LEDH's: the past posterior mean x_{k-1|k-1} (tracker.get_past_mean(), edh.py:213), from which
 * the shared linearisation trajectory etabar starts.  pf_ledh_step / pf_ledh_run therefore
 * refuse an EDH handle (PF_E_ARG); use pf_edh_step / pf_edh_run.
 *
 * Arithmetic is fp64 (the reference's).  Conventions (status codes, ownership, one handle =
 * one device + one stream, not re-entrant) are those of pf_engine.h.
 */
#ifndef PF_EDH_H
#define PF_EDH_H

#include <stdint.h>

#include "pf_ledh.h"

#ifdef __cplusplus
extern "C" {
#endif

/* EDHConfig.flow_integrator (edh.py:63): "rk4" (default) or "euler" (edh.py:271-280) */
#define PF_EDH_RK4 0
#define PF_EDH_EULER 1

typedef struct pf_edh_opts {
  int64_t n_particles;       /* EDHConfig.n_particles (edh.py:60) */
  int32_t n_lambda;          /* EDHConfig.n_lambda_steps (edh.py:61), clamped to >= 1 (edh.py:216) */
  double resample_ess_ratio; /* EDHConfig.resample_ess_ratio (edh.py:62); 0 disables resampling */
  uint64_t seed;             /* Philox key for PF_NOISE_DEVICE / device init / device resampling */
  int32_t device;
  int32_t integrator;        /* PF_EDH_RK4 | PF_EDH_EULER */
} pf_edh_opts;

/* EDHFlowPF.__init__ (edh.py:138-171): same model description as pf_ledh_create. */
pf_status pf_edh_create(const pf_model_desc* model, const pf_edh_opts* opts, pf_ledh_handle** out);

/* One flow step up to the weights (edh.py:185-297): P [nx][nx] = the tracker's predicted covariance
 * (symmetrised here, edh.py:197), xbar [nx] = its past mean x_{k-1|k-1} (edh.py:213), z [nz],
 * u [nx] or NULL, noise PF_NOISE_* with v [N][nx] for PF_NOISE_HOST.  info (nullable): ESS of the
 * normalised weights and the resample decision (edh.py:304-306), applied by pf_ledh_finish.
 * cond_S (nullable, [L][nz][nz]): S(lambda_j) for the condition-number diagnostics (edh.py:238-243). */
pf_status pf_edh_step(pf_ledh_handle* h, const double* P, const double* xbar, const double* z, const double* u,
                      int32_t noise, const double* v, pf_ledh_info* info, double* cond_S);

/* The whole T loop on the device with no host synchronisation inside T: Ps [T][nx][nx] tracker
 * covariances, Xbars [T][nx] the tracker's past means, Z [T][nz], U [T][nx] or NULL.  Noise
 * PF_NOISE_NONE, PF_NOISE_DEVICE (resampling uniforms from Philox) or PF_NOISE_HOST: the replayed
 * draws set by pf_ledh_set_run_replay for a run of exactly this T — step t's process noise V_t
 * [N][nx] and resampling uniform U_t, where U_t is read only on steps that resample, so the caller
 * lays the uniforms out with the decisions it expects and checks the returned flags against them.
 * A failed launch or grid-barrier timeout inside the run leaves the handle uninitialised
 * (PF_E_NOT_INITIALIZED on the next call).  Outputs as pf_ledh_run. */
pf_status pf_edh_run(pf_ledh_handle* h, const double* Ps, const double* Xbars, const double* Z, const double* U,
                     int64_t T, int32_t noise, double* means, double* covs, double* ess, uint8_t* flags);

/* 1 for a handle made by pf_edh_create. */
int32_t pf_edh_is_edh(pf_ledh_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* PF_EDH_H */
