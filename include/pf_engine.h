/*
 * pf_engine.h — C ABI of the MI355X SIR particle-filter engine (libpf_hip.so).
 *
 * Plain C types only (pointers + sizes); no torch / HIP types cross this line.
 * Every entry point returns a pf_status (PF_OK == 0); pf_last_error() gives a
 * thread-local message for the last failure.  Host arrays are caller-owned and
 * copied in/out; device buffers are owned by the handle.  One handle = one
 * device + one HIP stream, not re-entrant; separate handles may be driven from
 * separate threads.
 *
 * Each entry replaces a piece of the reference's Python filter
 * (/root/reference/models/particle_filter.py, cited "pf.py:LINE"); the Python
 * mirror particle_filters_amd/particle_filter.py binds them via ctypes (see
 * INTEGRATION.md for the binding a maintainer of the reference would add).
 */
#ifndef PF_ENGINE_H
#define PF_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t pf_status;
#define PF_OK 0
#define PF_E_NOT_INITIALIZED 1 /* -> AssertionError("Filter not initialized.") pf.py:142,231,252 */
#define PF_E_ARG 2             /* bad shape / argument -> ValueError */
#define PF_E_NOT_PD 3          /* Cholesky failed -> numpy.linalg.LinAlgError */
#define PF_E_HIP 4             /* HIP runtime error */
#define PF_E_UNSUPPORTED 5     /* model shape not compiled into this library */
#define PF_E_NAN 6             /* every particle weight zero or NaN (all-dead filter) -> FloatingPointError */
#define PF_E_RETRY 7           /* pf_run_device: the resident grid was not co-resident; nothing computed, state
                                  unchanged, the handle launches cooperatively from now on: run again */

/* g: transition kinds (pf.py:237 per-particle g(x,u)) */
#define PF_TRANS_LINEAR 0 /* x' = A x (+ u)                         params: A[nx*nx]         */
#define PF_TRANS_L96 1    /* one RK4 step of Lorenz-96              params: F, dt            */
/* h: observation kinds (pf.py:257 per-particle h(x)) */
#define PF_OBS_LINEAR 0   /* z = H x + c                            params: H[nz*nx], c[nz]  */
#define PF_OBS_EXP_HALF 1 /* z_k = beta_k exp(x_k / 2)   (nz==nx)   params: beta[nz]         */
#define PF_OBS_ACOUSTIC 2 /* z_s = sum_c psi/(|p_c-s|^2+d0) (nx=4C) params: psi, d0, sx[nz], sy[nz] */
#define PF_OBS_SV_EXACT 3 /* exact SV likelihood y_k ~ N(0, beta_k^2 e^{x_k}) (nz==nx) params: beta[nz];
                             log p = -x/2 - y^2 e^{-x}/(2 beta^2): test_dpf_vs_sv_simulator.py:60-97.
                             R is not used (pass any PD matrix, e.g. I). */
#define PF_OBS_BEARINGS 4 /* angles of a sensor at s: [atan2(x0-s0, x1-s1), atan2(x2-s2, |(x0,x1)-(s0,s1)|)]
                             (nz==2, nx>=3)                          params: s[3]
                             (SPF_results_reproduction_example2.ipynb cell 1 e2_measurement_function) */

#define PF_RESAMPLE_SYSTEMATIC 0 /* pf.py:146-171 */
#define PF_RESAMPLE_MULTINOMIAL 1 /* pf.py:173-186 (any other method string) */

#define PF_PRECISION_FP32 0
#define PF_PRECISION_FP64 1

typedef struct pf_model_desc {
  int32_t nx, nz;
  int32_t trans_kind, obs_kind;
  const double* trans_params; /* see PF_TRANS_* */
  int64_t n_trans_params;
  const double* obs_params;   /* see PF_OBS_* */
  int64_t n_obs_params;
  const double* Q; /* nx*nx process-noise covariance (pf.py:94) */
  const double* R; /* nz*nz measurement-noise covariance (pf.py:95) */
} pf_model_desc;

typedef struct pf_opts {
  int64_t n_particles;     /* Np (pf.py:96) */
  int32_t n_replicates;    /* independent filters batched in one launch (>= 1) */
  int32_t resample_method; /* PF_RESAMPLE_* (pf.py:98, 205-208) */
  double resample_thresh;  /* resample when Neff < thresh * Np (pf.py:97, 204) */
  int32_t regularize;      /* jitter 0.001*chol(Q) n after resampling (pf.py:99, 212-218) */
  int32_t precision;       /* PF_PRECISION_* : particle storage / arithmetic type */
  uint64_t seed;           /* Philox key; replicate r uses counter word r */
  int32_t device;          /* HIP device ordinal */
  int32_t replicate_base;  /* global id of local replicate 0: replicate r draws with counter
                              word replicate_base + r, so sharding replicates over GPUs gives
                              bitwise the same per-replicate results as one GPU */
  int32_t kernel_path;     /* PF_PATH_*: which step kernels serve the model */
} pf_opts;

#define PF_PATH_AUTO 0    /* the compiled shape's kernels when (nx, nz, g, h) is in the compiled list,
                             else the runtime-shape kernels */
#define PF_PATH_RUNTIME 1 /* always the runtime-shape kernels (pf_dyn.h): any nx, nz */

typedef struct pf_handle pf_handle;

/* Per-replicate posterior summary of one update (pf.py:262-268). */
typedef struct pf_update_info {
  double neff;     /* pre-resample 1/sum w^2 (pf.py:203) */
  double log_norm; /* log sum_i w_{t-1,i} exp(-quad_i/2): marginal-likelihood increment */
  int32_t resample; /* 1 if Neff < thresh*Np (the resample is applied by pf_resample) */
  int32_t _pad;
} pf_update_info;

const char* pf_last_error(void);
const char* pf_version(void);
int32_t pf_device_count(void);

/* ParticleFilter.__init__ (pf.py:79-107): validates the model, factorises R
 * (+1e-12 I) and Q (+1e-10 I / +1e-12 I fallbacks), allocates device state. */
pf_status pf_create(const pf_model_desc* model, const pf_opts* opts, pf_handle** out);
void pf_destroy(pf_handle* h);
/* Can the engine run (nx, nz, trans_kind, obs_kind)?  Any positive shape whose kinds fit
 * (EXP_HALF / SV_EXACT: nz == nx; ACOUSTIC: nx % 4 == 0; BEARINGS: nz == 2, nx >= 3). */
int32_t pf_model_supported(int32_t nx, int32_t nz, int32_t trans_kind, int32_t obs_kind);
/* Is the shape in the compiled (register-state) list, i.e. does PF_PATH_AUTO pick those kernels? */
int32_t pf_model_compiled(int32_t nx, int32_t nz, int32_t trans_kind, int32_t obs_kind);
/* PF_PATH_RUNTIME if the handle runs the runtime-shape kernels, else PF_PATH_AUTO. */
int32_t pf_kernel_path(pf_handle* h);
/* 1 if the handle's last fused step launch ran the persistent many-replicate kernel (k_step_stream:
 * fp32 scalar models with per-step replicate heads; PF_STREAM=0 turns it off), else 0.  Diagnostics. */
int32_t pf_last_step_streamed(pf_handle* h);

/* initialize (pf.py:110-132): particles ~ N(mean_r, cov_r), uniform weights.
 * mean [R][nx], cov [R][nx][nx]; replay_normals [R][N][nx] or NULL (device Philox). */
pf_status pf_initialize(pf_handle* h, const double* mean, const double* cov, const double* replay_normals);

/* predict (pf.py:223-237): x <- g(x, u) + chol(Q) n.  u [R][nx] or NULL;
 * replay_normals [R][N][nx] or NULL. */
pf_status pf_predict(pf_handle* h, const double* u, const double* replay_normals);

/* update, weighting half (pf.py:253-264 up to the resample decision).
 * z [R][nz]; info [R] out (nullable); mean [R][nx], cov [R][nx][nx] out (nullable):
 * the weighted posterior (the reported state when no resample happens). */
pf_status pf_update(pf_handle* h, const double* z, pf_update_info* info, double* mean, double* cov);

/* _resample, applying half (pf.py:204-218): replicates whose last update decided to
 * resample get their ancestors gathered (+ jitter); weights become uniform.
 * uniforms: NULL (device Philox) or [R] systematic U / [R][N] multinomial u;
 * jitter_normals [R][N][nx] or NULL.  mean/cov out (nullable): uniform-weight
 * statistics of the resampled set (pf.py:266-267), written for resampled replicates. */
pf_status pf_resample(pf_handle* h, const double* uniforms, const double* jitter_normals, double* mean,
                      double* cov);

/* Force a resample of the current (set_state) particles with their weights, whatever
 * Neff is: the applying half of ParticleFilter._resample(particles, weights) once the
 * caller has made the Neff test itself (pf.py:203-218).  uniforms / jitter as in
 * pf_resample (NULL = device Philox). */
pf_status pf_resample_state(pf_handle* h, const double* uniforms, const double* jitter_normals);

/* The device-resident T loop: for t in [0,T): step(Z[t], U[t]) — or update(Z[0]) first
 * when first_update_only (notebook driver, PF_VS_experiments.ipynb cell 7) — with no
 * host synchronisation inside T.  Z [T][R][nz]; U [T][R][nx] or NULL.
 * Outputs (host, nullable): means [T][R][nx] (post-resample when resampled, as the
 * reference's PFState.mean), covs [T][R][nx][nx] (any nx: the step records carry them for nx <= 4,
 * the device-loop covariance kernels of pf_cov.h for larger states), neff [T][R] (pre-resample),
 * flags [T][R], log_norm [T][R]. */
pf_status pf_run(pf_handle* h, const double* Z, const double* U, int64_t T, int32_t first_update_only,
                 double* means, double* covs, double* neff, uint8_t* flags, double* log_norm);

/* Same, with every array already in device memory (HBM-resident inputs and outputs;
 * Z/U in the engine precision).  No host copies, no synchronisation: returns after
 * enqueueing on the handle's stream.  flags are int32 [T][R]. */
pf_status pf_run_device(pf_handle* h, const void* dZ, const void* dU, int64_t T, int32_t first_update_only,
                        double* d_means, double* d_covs, double* d_neff, int32_t* d_flags,
                        double* d_log_norm);

/* State readout / injection.  particles [R][N][nx] (AoS like PFState.particles);
 * log_weights [R][N] normalised (log w); weights [R][N]. */
pf_status pf_get_particles(pf_handle* h, double* particles);
pf_status pf_get_weights(pf_handle* h, double* weights, double* log_weights);
pf_status pf_set_state(pf_handle* h, const double* particles, const double* weights);
int32_t pf_weights_uniform(pf_handle* h);

/* Philox position of the handle (SURVEY.md §5 checkpoint/resume; the reference's counterpart is
 * the NumPy Generator state behind self.rng, pf.py:100-101).  The next predict draws at `epoch`,
 * the next update reserves epoch + 1 for its resample; `ep_res` is the epoch of the resample the
 * last update decided (pending = 1 while it is not yet applied).  pf_set_rng_state moves the
 * handle to a position (seed = Philox key, replicate_base = counter word of replicate 0);
 * `pending` is ignored on set. */
typedef struct pf_rng_state {
  uint64_t seed;
  uint32_t epoch;
  uint32_t ep_res;
  int32_t replicate_base;
  int32_t pending;
} pf_rng_state;
pf_status pf_get_rng_state(pf_handle* h, pf_rng_state* out);
pf_status pf_set_rng_state(pf_handle* h, const pf_rng_state* in);

/* Bit-exact checkpoint / resume of the whole filter state at a step boundary (a decided
 * resample is applied first): particles and UNNORMALISED log-weights in the engine precision,
 * the tile records, the systematic-CDF prefix, the resident kernel's entry header and the
 * Philox position.  Restoring into a handle created with the same model and options (shape,
 * Np, replicates, precision, resample method) continues bitwise as the original would have.
 * The blob is opaque host memory of pf_checkpoint_bytes(h) bytes. */
int64_t pf_checkpoint_bytes(pf_handle* h);
pf_status pf_checkpoint(pf_handle* h, void* buf, int64_t nbytes);
pf_status pf_restore(pf_handle* h, const void* buf, int64_t nbytes);

/* Weighted mean/cov of the current state, exact two-pass (np.average / np.cov
 * aweights, bias=True; pf.py:266-267), any nx.  mean [R][nx], cov [R][nx][nx]. */
pf_status pf_moments(pf_handle* h, double* mean, double* cov);

/* Standalone resampling of caller weights (pf.py:146-186 _systematic_resample /
 * _multinomial_resample).  w [N] normalised; method PF_RESAMPLE_*; systematic uses U,
 * multinomial uses uniforms [N].  idx [N] int64 out. */
pf_status pf_resample_indices(int32_t device, int32_t method, const double* w, int64_t N, double U,
                              const double* uniforms, int64_t* idx);

/* Measurement hooks for bench.py: the handle's HIP stream (hipStream_t as void*),
 * synchronisation, and per-launch device durations of `steps` step-kernels timed
 * with HIP events on that stream (ms_out [steps]). */
void* pf_stream(pf_handle* h);
pf_status pf_synchronize(pf_handle* h);
pf_status pf_profile_steps(pf_handle* h, const void* dZ, int64_t steps, float* ms_out);
/* 1 if the last pf_run / pf_run_device ran as the register-resident whole-run
 * kernel (one launch for all T steps: scalar fp32 models, systematic resampling,
 * grid co-resident), 0 if as the launch-per-step loop.  PF_RESIDENT=0 in the
 * environment forces the launch-per-step loop. */
int32_t pf_last_run_resident(pf_handle* h);
/* 1 if the last pf_run / pf_run_device ran as the persistent fp64 whole-run kernel (k_persist: one
 * launch for the T steps, the tail and the statistics; scalar fp64 models, systematic resampling,
 * grid co-resident; bitwise the launch-per-step loop), 0 otherwise.  Opt-in: PF_PERSIST=1 in the
 * environment (it is not faster than the launch-per-step loop at N = 1e6).  No reference counterpart
 * (replaces the per-step calls of models/particle_filter.py:223-269 as the resident kernel does). */
int32_t pf_last_run_persistent(pf_handle* h);
/* Uninitialised-LDS test hooks (tests/test_gpu_lds_poison.py; no reference counterpart):
 * pf_test_lds_poison fills the whole 160 KB of LDS of every CU with 0xFFFFFFFF (NaN in fp32 and
 * fp64) on `stream` (a hipStream_t); with PF_TEST_HOOKS=1 and PF_TEST_LDS_POISON=1 in the
 * environment the engine does the same before every launch of its LDS-staging step, flow, EKF and
 * covariance kernels.  pf_test_lds_probe launches pf_test_lds_probe_blocks() workgroups that count
 * the words of their uninitialised LDS not holding that pattern (out [blocks], waits). */
pf_status pf_test_lds_poison(void* stream);
int32_t pf_test_lds_probe_blocks(void);
int64_t pf_test_lds_poison_count(void);  /* poison launches the engine's hook has made so far */
pf_status pf_test_lds_probe(void* stream, int32_t* out);
/* Live kernel timing for the bench: when on, every pf_run_device records HIP events on
 * the handle's stream right before its first and after its last filter kernel;
 * pf_last_run_ms waits for the last run and returns the device time between them. */
pf_status pf_set_timing(pf_handle* h, int32_t on);
pf_status pf_last_run_ms(pf_handle* h, float* ms);
/* Verification trace of the register-resident kernel (tests; the shipped kernel instance is not
 * touched: a second instance with the trace stores runs while a trace is set).  pf_set_trace
 * allocates room for T_cap steps (0 frees it).  While set, every resident run records, for each
 * of its first T_cap steps, the state its verification accepted - after any rollback and
 * recomputation inside the launch: the predicted particles and pre-resample log-weights (fp32,
 * any uniform frame), and on a resample step the ancestor index of every output slot (-1
 * elsewhere).  pf_get_trace copies step t (of the last run) of replicate r: x, l, anc [N]
 * (nullable), and resets that step's ancestors to -1; PF_E_ARG when the last run did not execute
 * as the resident kernel (a launch-per-step run records no trace). */
pf_status pf_set_trace(pf_handle* h, int64_t T_cap);
pf_status pf_get_trace(pf_handle* h, int64_t t, int32_t r, float* x, float* l, int32_t* anc);
/* Geometry of the step launch: tiles per replicate, tile size, dynamic LDS bytes. */
pf_status pf_geometry(pf_handle* h, int32_t* G, int32_t* tile, int32_t* lds_bytes);

#ifdef __cplusplus
}
#endif
#endif /* PF_ENGINE_H */
