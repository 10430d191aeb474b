/*
 * pf_diag.h — particle-degeneracy diagnostics on the GPU (libpf_hip.so).
 *
 * Replaces the host diagnostics of the reference's degeneracy study
 * (/root/reference/notebooks/particle_filter_NLNGSSM.ipynb cell 5, cited "diag:LINE" =
 * line within that cell): compute_weight_entropy 5-19, compute_gini_coefficient 22-36,
 * count_unique_particles 39-58, compute_diagnostics 61-91 (ESS = 1 / sum w^2 as
 * ParticleFilter.effective_sample_size, particle_filter.py:134-144; posterior spread =
 * trace of the state covariance).  The Python mirror is particle_filters_amd/diagnostics.py.
 *
 * The state entries read the particles and weights where they live (HBM) — nothing crosses
 * PCIe but the result.  Conventions are those of pf_engine.h.
 */
#ifndef PF_DIAG_H
#define PF_DIAG_H

#include <stdint.h>

#include "pf_engine.h"
#include "pf_ledh.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pf_diagnostics {
  double ess;              /* 1 / sum w^2 */
  double entropy;          /* -sum (w + 1e-300) log(w + 1e-300) / log N  (normalised; N > 1) (diag:5-19) */
  double entropy_raw;      /* the same without the / log N */
  double gini;             /* (2 sum_i i w_(i)) / (N sum w) - (N + 1) / N, ascending w, i = 1..N (diag:22-36) */
  double max_weight;
  double posterior_spread; /* trace of the weighted covariance of the particles (NaN without particles) */
  int64_t n_unique;        /* distinct rows of round(x / tol) * tol (diag:39-58); -1 without particles */
} pf_diagnostics;

/* Host arrays: weights [N] (normalised), particles [N][nx] or NULL.  cov [nx][nx] or NULL:
 * when given, posterior_spread = trace(cov) (as compute_diagnostics reads state.cov), otherwise
 * it is the weighted covariance trace of the particles. */
pf_status pf_diagnostics_host(int32_t device, const double* weights, const double* particles, int64_t N, int32_t nx,
                              double tol, const double* cov, pf_diagnostics* out);

/* The SIR handle's current state, one record per replicate: out [R]. */
pf_status pf_state_diagnostics(pf_handle* h, double tol, pf_diagnostics* out);

/* An LEDH / EDH handle's current state. */
pf_status pf_ledh_diagnostics(pf_ledh_handle* h, double tol, pf_diagnostics* out);

#ifdef __cplusplus
}
#endif
#endif /* PF_DIAG_H */
