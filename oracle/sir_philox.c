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

/*
 * One step of the filter from a given state, compared with an engine's record of the same
 * step (the verification trace of the register-resident kernel, include/pf_engine.h
 * pf_get_trace).  Oracle side: pf.py:223-269 + _resample pf.py:188-220 in fp64 on the
 * engine's Philox draws (predict epoch c->epoch, resample epoch c->epoch + 1), started from
 * x0 / w0 (the engine's state before the step, w0 normalised).  Engine side: xe [N] predicted
 * particles, le [N] pre-resample log-weights (fp32, any uniform frame), anc [N] the ancestor of
 * every slot when the engine resampled (NULL otherwise), and the step's reported Neff / flag /
 * mean / variance (post-resample moments when it resampled, pf.py:266-267).  Every quantity of
 * c's "measured" block is filled in; the tolerances are the caller's.  Returns 0, -1 when an
 * allocation failed.
 */
typedef struct pfo_step_check {
  /* in */
  int64_t N;
  uint64_t seed;
  uint32_t rep, epoch;
  double thresh;
  int32_t bm24, regularize;
  double u;  /* control input of the step (0: none) */
  double z;
  double neff_e, mean_e, var_e;
  int32_t flag_e, _pad0;
  /* measured */
  double dx_pre;       /* max |xe - x_oracle| after predict */
  double mean_abs_x;   /* E_w |x_oracle| (scale of the state) */
  double tv_w;         /* total-variation distance of the normalised weights */
  double dcdf;         /* max |cdf_e - cdf_o| (fp64 cumsums of both weight sets) */
  double lmag;         /* E_w |log-likelihood| (oracle weights) */
  double eps_w;        /* E_w of the per-particle fp32 rounding bound of the engine's weights */
  double neff_o, neff_rel;
  int32_t flag_o, near_threshold;
  double U;            /* systematic uniform of the step */
  int64_t n_anc_bad;   /* slots with an ancestor out of range / unwritten / not monotone */
  int64_t n_anc_self_diff, n_anc_oracle_diff;
  double max_margin_self, max_margin_oracle;  /* distance of a differing slot's position to its
                                                 ancestor's interval (engine's own / oracle CDF) */
  double dmean, dvar;  /* engine mean / variance vs the oracle's set under the engine's decision
                          (and ancestors) */
  double dmean_oracle; /* vs the oracle's own ancestors */
  double mean_o, var_o;
} pfo_step_check;

static double dll_dz(const pfo_scalar_model* m, double x, double z) {
  if (m->obs == 3) return -z * exp(-x) / (m->hc * m->hc);
  const double hp = m->obs == 0 ? m->hH * x + m->hc : m->hc * exp(0.5 * x);
  return -(z - hp) / (m->lr * m->lr);
}

static double dll_dx(const pfo_scalar_model* m, double x, double z) {
  if (m->obs == 3) {
    const double b2 = m->hc * m->hc;
    return -0.5 * (1.0 - z * z * exp(-x) / b2);
  }
  const double hp = m->obs == 0 ? m->hH * x + m->hc : m->hc * exp(0.5 * x);
  const double dh = m->obs == 0 ? m->hH : 0.5 * hp;
  return (z - hp) / (m->lr * m->lr) * dh;
}

/* distance of pos to the interval [lo, hi) of ancestor a in cdf (0 inside) */
static double interval_dist(const double* cdf, int64_t a, double pos) {
  const double lo = a > 0 ? cdf[a - 1] : 0.0, hi = cdf[a];
  if (pos < lo) return lo - pos;
  if (pos >= hi) return pos - hi;
  return 0.0;
}

int pfo_sir_scalar_check_step(const pfo_scalar_model* m, pfo_step_check* c, const double* x0, const double* w0,
                              const float* xe, const float* le, const int32_t* anc) {
  const int64_t N = c->N;
  double* xo = (double*)malloc((size_t)N * sizeof(double));
  double* wo = (double*)malloc((size_t)N * sizeof(double));
  double* we = (double*)malloc((size_t)N * sizeof(double));
  double* tmp = (double*)malloc((size_t)N * sizeof(double));
  double* ll = (double*)malloc((size_t)N * sizeof(double));
  if (!xo || !wo || !we || !tmp || !ll) {
    free(xo); free(wo); free(we); free(tmp); free(ll);
    return -1;
  }
  /* predict (pf.py:232-237) */
  pfo_normals(c->seed, N, c->rep, c->epoch, 2u, c->bm24, tmp);
  double dx = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    xo[i] = (m->a * x0[i] + c->u) + tmp[i] * m->lq;
    const double d = fabs((double)xe[i] - xo[i]);
    if (d > dx || isnan(d)) dx = d;
  }
  c->dx_pre = dx;
  /* update (pf.py:253-262) and the engine's weights from its own log-weights (fp64 softmax) */
  double mo = -INFINITY, me = -INFINITY;
  for (int64_t i = 0; i < N; ++i) {
    ll[i] = -0.5 * quad_of(m, xo[i], c->z);
    wo[i] = log(w0[i] + 1e-300) + ll[i];
    if (wo[i] > mo) mo = wo[i];
    if ((double)le[i] > me) me = (double)le[i];
  }
  double so = 0.0, se = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    wo[i] = exp(wo[i] - mo);
    so += wo[i];
    we[i] = (le[i] > -INFINITY) ? exp((double)le[i] - me) : 0.0;
    se += we[i];
  }
  double tv = 0.0, w2 = 0.0, lmag = 0.0, eps = 0.0, ax = 0.0, co = 0.0, ce = 0.0, dcdf = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    wo[i] /= so;
    we[i] /= se;
    tv += fabs(we[i] - wo[i]);
    w2 += wo[i] * wo[i];
    lmag += wo[i] * fabs(ll[i]);
    ax += wo[i] * fabs(xo[i]);
    /* the fp32 rounding bound of the engine's log-weight of particle i: 8 fp32 half-ulps (2^-21
       relative) of the log-weight and log-likelihood it is built from (the carried log-weight's
       shift, the likelihood's few fp32 operations, the add), the fp32 observation carried through
       the likelihood's slope in z, and the predicted particle's own rounding carried through its
       slope in x */
    const double ep = ldexp(1.0 + fabs((double)le[i]) + fabs(ll[i]), -21) +
                      ldexp(fabs(dll_dz(m, xo[i], c->z)) * fabs(c->z), -23) +
                      fabs(dll_dx(m, xo[i], c->z)) * fabs((double)xe[i] - xo[i]);
    eps += wo[i] * ep;
    co += wo[i];
    ce += we[i];
    const double d = fabs(ce - co);
    if (d > dcdf) dcdf = d;
  }
  c->tv_w = 0.5 * tv;
  c->dcdf = dcdf;
  c->lmag = lmag;
  c->eps_w = eps;
  c->mean_abs_x = ax;
  c->neff_o = 1.0 / w2;
  c->neff_rel = fabs(c->neff_e / c->neff_o - 1.0);
  c->flag_o = c->neff_o < c->thresh * (double)N;
  c->near_threshold = fabs(c->neff_o - c->thresh * (double)N) / (double)N < 1e-3;
  c->n_anc_bad = c->n_anc_self_diff = c->n_anc_oracle_diff = 0;
  c->max_margin_self = c->max_margin_oracle = 0.0;
  c->U = pfo_uniform53(c->seed, 0, c->rep, c->epoch + 1u);
  if (c->flag_e && anc) {
    /* the post-resample set under the engine's ancestors (+ the jitter, pf.py:212-218) */
    double* cdf_o = tmp;
    double* cdf_s = ll;
    double a = 0.0, b = 0.0;
    for (int64_t i = 0; i < N; ++i) {
      a += wo[i];
      cdf_o[i] = a;
      b += we[i];
      cdf_s[i] = b;
    }
    cdf_o[N - 1] = 1.0;
    cdf_s[N - 1] = 1.0;
    double* jit = NULL;
    if (c->regularize) {
      jit = (double*)malloc((size_t)N * sizeof(double));
      if (!jit) {
        free(xo); free(wo); free(we); free(tmp); free(ll);
        return -1;
      }
      pfo_normals(c->seed, N, c->rep, c->epoch + 1u, 3u, c->bm24, jit);
    }
    double sf = 0.0, so2 = 0.0;
    int64_t jo = 0, js = 0, prev = 0;
    for (int64_t i = 0; i < N; ++i) {
      const double pos = (c->U + (double)i) / (double)N;
      while (jo < N - 1 && !(pos < cdf_o[jo])) ++jo; /* searchsorted(cdf, pos, 'right') */
      while (js < N - 1 && !(pos < cdf_s[js])) ++js;
      int64_t ai = anc[i];
      if (ai < 0 || ai >= N || ai < prev) {
        ++c->n_anc_bad;
        ai = jo;
      } else {
        prev = ai;
      }
      if (ai != js) {
        ++c->n_anc_self_diff;
        const double d = interval_dist(cdf_s, ai, pos);
        if (d > c->max_margin_self) c->max_margin_self = d;
      }
      if (ai != jo) {
        ++c->n_anc_oracle_diff;
        const double d = interval_dist(cdf_o, ai, pos);
        if (d > c->max_margin_oracle) c->max_margin_oracle = d;
      }
      const double j = jit ? jit[i] * m->lj : 0.0;
      sf += xo[ai] + j;
      so2 += xo[jo] + j;
      we[i] = xo[ai] + j; /* reuse: the forced set */
    }
    const double mf = sf / (double)N;
    double vf = 0.0;
    for (int64_t i = 0; i < N; ++i) vf += (we[i] - mf) * (we[i] - mf);
    vf /= (double)N;
    c->mean_o = mf;
    c->var_o = vf;
    c->dmean = fabs(c->mean_e - mf);
    c->dvar = fabs(c->var_e - vf);
    c->dmean_oracle = fabs(c->mean_e - so2 / (double)N);
    free(jit);
  } else {
    /* no resample on the engine's side: the weighted predicted set (pf.py:266-267) */
    double sw = 0.0, sx = 0.0;
    for (int64_t i = 0; i < N; ++i) {
      sw += wo[i];
      sx += wo[i] * xo[i];
    }
    const double mean = sx / sw;
    double v = 0.0;
    for (int64_t i = 0; i < N; ++i) v += wo[i] * (xo[i] - mean) * (xo[i] - mean);
    v /= sw;
    c->mean_o = mean;
    c->var_o = v;
    c->dmean = c->dmean_oracle = fabs(c->mean_e - mean);
    c->dvar = fabs(c->var_e - v);
  }
  free(xo); free(wo); free(we); free(tmp); free(ll);
  return 0;
}
