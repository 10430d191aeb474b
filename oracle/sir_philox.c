/*
 * sir_philox.c — CPU restatement of the reference SIR filter for scalar state
 * models, driven by the engine's counter-based Philox draws.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline / rmse_vs_ref legs (through oracle/sir_philox.py),
 * never by particle_filters_amd/.  It is the checker, not the product.
 *
 * Algorithm: /root/reference/models/particle_filter.py (cited pf.py:LINE), fp64,
 * the same operations as oracle/pf_oracle.py:SIROracle (which is pinned bit for
 * bit to the reference's own outputs, tests/test_oracle_golden.py):
 *   initialize  pf.py:110-132  x = mean + chol(cov + 1e-10) n,  w = 1/N
 *   predict     pf.py:223-237  x = g(x, u) + chol(Q) n
 *   update      pf.py:239-269  logw = log(w + 1e-300) - quad/2, max-shifted normalise,
 *                              Neff = 1/sum w^2, resample if Neff < thresh N,
 *                              mean / biased weighted variance
 *   _resample   pf.py:188-220  systematic: searchsorted(cdf, (U+i)/N, 'right'), cdf[-1] = 1
 *                              (pf.py:146-171); multinomial: searchsorted(cdf/cdf[-1], u_i)
 *                              (pf.py:173-186); jitter 0.001 chol(Q) n (pf.py:212-218)
 * The random numbers are the engine's instead of NumPy's PCG64 stream
 * (particle_filters_amd/csrc/philox.h, restated in oracle/philox.py):
 *   normal of particle i, epoch e, stream s = Box-Muller component (i & 3) of
 *   Philox4x32-10(counter = (i >> 2, replicate, e, s), key = seed);
 *   systematic U / multinomial u_i = u53 of Philox((i, replicate, e, 4));
 *   epochs: initialize e0 - 1, step t predicts at e0 + 2t - fo and resamples at
 *   e0 + 2t + 1 - fo (fo = 1 when the first step is update-only).
 * bm24 = 1 maps the radius uniform from 24 bits (the fp32 engine's Box-Muller),
 * bm24 = 0 from 32 bits (the fp64 engine's); the arithmetic is fp64 either way.
 *
 * Observation kinds (the engine's PF_OBS_*):
 *   0 LINEAR   z = hH x + hc, quad = ((z - h)/lr)^2 with lr = sqrt(R + 1e-12) (pf.py:107)
 *   1 EXP_HALF z = hc exp(x/2), quad as LINEAR
 *   3 SV_EXACT log p(y|x) = -x/2 - y^2 exp(-x) / (2 beta^2) (+ const), beta = hc
 *              (tests/integration_tests/test_dpf_vs_sv_simulator.py:60-97); quad is
 *              replaced by -2 log p, the Gaussian constants dropped as pf.py drops them.
 *
 * Determinism: per-particle loops may run on several OpenMP threads; every
 * reduction is a sum over fixed 4096-particle blocks combined in block order,
 * so results do not depend on the thread count.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLK 4096

static void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t out[4]) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

void pfo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  philox(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1], out);
}

static double radius(uint32_t a, int bm24) {
  const double u = bm24 ? ((double)(a >> 8) + 1.0) * (1.0 / 16777216.0) : ((double)a + 1.0) * (1.0 / 4294967296.0);
  return sqrt(-2.0 * log(u));
}

/* the 4 normals of one Philox group (philox.h box_muller4 / box_muller4_f64) */
static void normal4(uint64_t seed, uint32_t group, uint32_t rep, uint32_t ep, uint32_t stream, int bm24, double v[4]) {
  uint32_t r[4];
  philox(group, rep, ep, stream, (uint32_t)seed, (uint32_t)(seed >> 32), r);
  const double r0 = radius(r[0], bm24), r1 = radius(r[2], bm24);
  const double a0 = (double)(r[1] >> 8) * (2.0 / 16777216.0) * 3.14159265358979323846, a1 = (double)(r[3] >> 8) * (2.0 / 16777216.0) * 3.14159265358979323846;
  v[0] = r0 * cos(a0);
  v[1] = r0 * sin(a0);
  v[2] = r1 * cos(a1);
  v[3] = r1 * sin(a1);
}

double pfo_uniform53(uint64_t seed, uint32_t index, uint32_t rep, uint32_t ep) {
  uint32_t r[4];
  philox(index, rep, ep, 4u, (uint32_t)seed, (uint32_t)(seed >> 32), r);
  const uint64_t a = r[0] >> 5, b = r[1] >> 6;
  return (double)((a << 26) | b) * (1.0 / 9007199254740992.0);
}

/* first n normals of (rep, epoch, stream) in flat order (oracle/philox.py normals) */
void pfo_normals(uint64_t seed, int64_t n, uint32_t rep, uint32_t ep, uint32_t stream, int bm24, double* out) {
  const int64_t groups = (n + 3) / 4;
#pragma omp parallel for schedule(static)
  for (int64_t g = 0; g < groups; ++g) {
    double v[4];
    normal4(seed, (uint32_t)g, rep, ep, stream, bm24, v);
    for (int k = 0; k < 4; ++k)
      if (4 * g + k < n) out[4 * g + k] = v[k];
  }
}

typedef struct pfo_scalar_model {
  double a;       /* g(x) = a x (+ u) */
  double lq;      /* chol(Q) (+1e-10 fallback, pf.py:232-235) */
  double lj;      /* 0.001 chol(Q) (+1e-12 fallback, pf.py:213-217) */
  int32_t obs;    /* 0 LINEAR, 1 EXP_HALF, 3 SV_EXACT */
  int32_t _pad;
  double hH, hc;  /* LINEAR: h = hH x + hc; EXP_HALF: h = hc exp(x/2); SV_EXACT: beta = hc */
  double lr;      /* chol(R + 1e-12) */
} pfo_scalar_model;

typedef struct pfo_run_opts {
  int64_t N, T;
  uint64_t seed;
  uint32_t rep, ep0; /* ep0: the handle's epoch at the first step (initialize used ep0 - 1) */
  double thresh;
  int32_t method;    /* 0 systematic, 1 multinomial */
  int32_t regularize;
  int32_t bm24;
  int32_t first_update_only;
  int32_t init;      /* 1: initialize(mean0, var0) first (epoch ep0 - 1); 0: start from x_io / w_io */
  int32_t _pad;
  double mean0, var0;
} pfo_run_opts;

static double quad_of(const pfo_scalar_model* m, double x, double z) {
  if (m->obs == 3) {  /* -2 log p(y|x) up to a constant */
    const double b2 = m->hc * m->hc;
    return x + z * z * exp(-x) / b2;
  }
  const double hp = m->obs == 0 ? m->hH * x + m->hc : m->hc * exp(0.5 * x);
  const double y = (z - hp) / m->lr;
  return y * y;
}

/* sum over fixed blocks in block order (thread-count independent) */
static double blocked_sum(const double* v, int64_t n, double* part) {
  const int64_t nb = (n + BLK - 1) / BLK;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nb; ++b) {
    double s = 0.0;
    const int64_t e = (b + 1) * BLK < n ? (b + 1) * BLK : n;
    for (int64_t i = b * BLK; i < e; ++i) s += v[i];
    part[b] = s;
  }
  double s = 0.0;
  for (int64_t b = 0; b < nb; ++b) s += part[b];
  return s;
}

/*
 * Run T steps.  x_io [N] / w_io [N]: final particles / weights out (and the start
 * state in when opts->init == 0).  Z [T] (and U [T] or NULL).  forced [T] or NULL:
 * when given, step t resamples iff forced[t] != 0 (decision teacher-forcing; the
 * filter's own Neff test is still reported in neff_out).  Outputs [T], nullable:
 * means, vars (reported state, post-resample when resampled, pf.py:266-267),
 * neff (pre-resample 1/sum w^2), flags (decision taken), lse (log sum_i w_{t-1,i}
 * exp(-quad_i/2)).  Returns 0, or 1 + t when step t had no finite weight.
 */
int64_t pfo_sir_scalar_run(const pfo_scalar_model* m, const pfo_run_opts* o, const double* Z, const double* U,
                           const int32_t* forced, double* x_io, double* w_io, double* means, double* vars,
                           double* neff_out, int32_t* flags, double* lse_out) {
  const int64_t N = o->N, nb = (N + BLK - 1) / BLK;
  double* lw = (double*)malloc((size_t)N * sizeof(double));
  double* tmp = (double*)malloc((size_t)N * sizeof(double));
  double* cdf = (double*)malloc((size_t)N * sizeof(double));
  double* part = (double*)malloc((size_t)nb * sizeof(double));
  double* bmax = (double*)malloc((size_t)nb * sizeof(double));
  int64_t status = 0;
  if (!lw || !tmp || !cdf || !part || !bmax) {
    status = -1;
    goto done;
  }
  const int fo = o->first_update_only ? 1 : 0;
  if (o->init) { /* pf.py:127-130 */
    const double lc = sqrt(o->var0 + 1e-10);
    pfo_normals(o->seed, N, o->rep, o->ep0 - 1, 1u, o->bm24, tmp);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) {
      x_io[i] = tmp[i] * lc + o->mean0;
      w_io[i] = 1.0 / (double)N;
    }
  }
  for (int64_t t = 0; t < o->T; ++t) {
    const uint32_t ep_pred = o->ep0 + (uint32_t)(2 * t) - (uint32_t)fo, ep_res = ep_pred + 1u;
    const double z = Z[t];
    if (!(fo && t == 0)) { /* predict, pf.py:232-237 */
      pfo_normals(o->seed, N, o->rep, ep_pred, 2u, o->bm24, tmp);
      const double u = U ? U[t] : 0.0;
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < N; ++i) x_io[i] = (m->a * x_io[i] + u) + tmp[i] * m->lq;
    }
    /* update, pf.py:253-261: logw = log(w + 1e-300) - quad / 2 */
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; ++b) {
      double mx = -INFINITY;
      const int64_t e = (b + 1) * BLK < N ? (b + 1) * BLK : N;
      for (int64_t i = b * BLK; i < e; ++i) {
        lw[i] = log(w_io[i] + 1e-300) - 0.5 * quad_of(m, x_io[i], z);
        if (lw[i] > mx) mx = lw[i];
      }
      bmax[b] = mx;
    }
    double mx = -INFINITY;
    for (int64_t b = 0; b < nb; ++b)
      if (bmax[b] > mx) mx = bmax[b];
    if (!(mx > -INFINITY) || isnan(mx)) {
      status = 1 + t;
      goto done;
    }
    /* lse increment: log sum_i w_prev_i exp(-quad_i / 2) (the log(w + 1e-300) carry) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) tmp[i] = exp(lw[i] - mx);
    const double s = blocked_sum(tmp, N, part);
    const double lse = mx + log(s);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) w_io[i] = exp(lw[i] - lse); /* pf.py:262 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) tmp[i] = w_io[i] * w_io[i];
    const double neff = 1.0 / blocked_sum(tmp, N, part); /* pf.py:203 */
    const int dec = forced ? (forced[t] != 0) : (neff < o->thresh * (double)N); /* pf.py:204 */
    if (dec) {
      /* cdf = cumsum(w) (serial: the prefix order is the reference's) */
      double c = 0.0;
      for (int64_t i = 0; i < N; ++i) {
        c += w_io[i];
        cdf[i] = c;
      }
      double* xs = lw; /* reuse: ancestors' values */
      if (o->method == 0) { /* systematic, pf.py:146-171 */
        cdf[N - 1] = 1.0;
        const double Us = pfo_uniform53(o->seed, 0, o->rep, ep_res);
        /* two-pointer walk of the reference loop == searchsorted(cdf, pos, 'right') */
        int64_t j = 0;
        for (int64_t i = 0; i < N; ++i) {
          const double pos = (Us + (double)i) / (double)N;
          while (j < N - 1 && !(pos < cdf[j])) ++j;
          xs[i] = x_io[j];
        }
      } else { /* multinomial, pf.py:173-186: choice(N, N, p=w) */
        const double tot = cdf[N - 1];
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) {
          const double u = pfo_uniform53(o->seed, (uint32_t)i, o->rep, ep_res);
          int64_t lo = 0, hi = N; /* first j with cdf[j]/tot > u */
          while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (cdf[mid] / tot > u) hi = mid;
            else lo = mid + 1;
          }
          xs[i] = x_io[lo < N ? lo : N - 1];
        }
      }
      if (o->regularize) { /* pf.py:212-218 */
        pfo_normals(o->seed, N, o->rep, ep_res, 3u, o->bm24, tmp);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < N; ++i) xs[i] += tmp[i] * m->lj;
      }
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < N; ++i) {
        x_io[i] = xs[i];
        w_io[i] = 1.0 / (double)N;
      }
    }
    /* pf.py:266-267 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) tmp[i] = w_io[i] * x_io[i];
    const double sw = blocked_sum(w_io, N, part); /* np.average divides by sum(w) */
    const double mean = blocked_sum(tmp, N, part) / sw;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i) tmp[i] = w_io[i] * (x_io[i] - mean) * (x_io[i] - mean);
    const double var = blocked_sum(tmp, N, part) / sw;
    if (means) means[t] = mean;
    if (vars) vars[t] = var;
    if (neff_out) neff_out[t] = neff;
    if (flags) flags[t] = dec;
    if (lse_out) lse_out[t] = lse;
  }
done:
  free(lw);
  free(tmp);
  free(cdf);
  free(part);
  free(bmax);
  return status;
}
