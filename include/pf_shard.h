/*
 * pf_shard.h — within-filter sharding of one SIR filter over several GPUs (libpf_hip.so).
 *
 * ONE ParticleFilter (/root/reference/models/particle_filter.py, "pf.py:LINE")
 * whose N_total particles do not fit one GPU is split into W equal shards, one pf_handle per
 * rank.  Every rank runs the same call sequence; between the calls the host orchestrator
 * (particle_filters_amd/sharded.py) exchanges a few doubles per shard (log normaliser, Neff,
 * weighted moments) and, on resample steps, migrates particles so that rank d ends up with the
 * global systematic-resampling slots [d N_loc, (d+1) N_loc):
 *
 *   pf_initialize / pf_predict   as usual (the handle draws the Philox normals of its GLOBAL
 *                                particle indices: a W-shard filter sees the noise of the
 *                                unsharded one)
 *   pf_shard_update              weights with the GLOBAL normaliser of the previous weights
 *                                (pf.py:254-261); returns this shard's lse / Neff / moments
 *   host                         lse = logsumexp_g lse_g, W_g = e^(lse_g - lse), Neff =
 *                                1 / sum_g W_g^2 / Neff_g, decision Neff < thresh N_total
 *                                (pf.py:198-203), shard boundaries B_g = prefix of W_g
 *   pf_shard_offspring           rows of the global slots [a, a+n) this shard's CDF segment owns
 *                                (pf.py:146-171 with positions (U + i) / N_total)
 *   exchange                     rows to the owning ranks (RCCL / gloo point-to-point)
 *   pf_shard_adopt               the received N_loc rows become the state, uniform weights,
 *                                optional 0.001 chol(Q) jitter (pf.py:212-218)
 *
 * Systematic resampling only.  Conventions are those of pf_engine.h.
 */
#ifndef PF_SHARD_H
#define PF_SHARD_H

#include <stdint.h>

#include "pf_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Make h (R = 1, systematic, N_loc = its n_particles) shard `rank` of a filter of n_total =
 * W * N_loc particles: its particle i is global particle rank * N_loc + i.  Call before
 * pf_initialize.  Device-RNG draws of a scalar-state shard need N_loc % 4 == 0 (its 4-particle
 * chunks must align with the Philox groups); host-replayed draws take any N_loc. */
pf_status pf_shard_configure(pf_handle* h, int64_t n_total, int32_t rank);

typedef struct pf_shard_stats {
  double lse;   /* log sum_i exp(l_i) of this shard's unnormalised log weights */
  double neff;  /* (sum w)^2 / sum w^2 of this shard's weights */
  double U;     /* the systematic offset the resample of this update would use (same on every rank) */
} pf_shard_stats;

/* update(z) on the shard (pf.py:239-263) without the resample decision.  lse_prev: the global
 * log normaliser of the previous weights (the host's logsumexp of the shards' lse), ignored when
 * the previous weights are uniform.  mean [nx], cov [nx][nx] (nullable): this shard's weighted
 * moments under its own normalised weights. */
pf_status pf_shard_update(pf_handle* h, const double* z, double lse_prev, pf_shard_stats* st, double* mean,
                          double* cov);

/* The particles of global systematic slots [a, a + n): positions (U + i) / n_total mapped into
 * this shard's CDF segment [lo, lo + mass) of the global CDF and searched in its own normalised
 * CDF.  out: device buffer of n rows [n][nx] in the handle's precision (float / double). */
pf_status pf_shard_offspring(pf_handle* h, double U, double lo, double mass, int64_t a, int64_t n, void* out);

/* The resampled shard: rows [N_loc][nx] (device, handle precision) become the particles in slot
 * order, weights uniform, + 0.001 chol(Q) jitter when the filter regularises: jitter [N_loc][nx]
 * host normals of this shard's slots (host replay of the reference's draw stream), or NULL for
 * the device Philox draws of the global slot indices.  mean [nx], cov [nx][nx] (nullable):
 * moments of the adopted particles. */
pf_status pf_shard_adopt(pf_handle* h, const void* rows, const double* jitter, double* mean, double* cov);

#ifdef __cplusplus
}
#endif
#endif /* PF_SHARD_H */
