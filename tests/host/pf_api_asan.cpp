// Host-side sanitizer driver of the C ABI (include/pf_engine.h): the engine's host code built with
// AddressSanitizer + UndefinedBehaviorSanitizer (host only: `make -C particle_filters_amd/csrc asan`),
// linked into this executable, driven through the entry points the reference's Python filter maps
// to (pf.py:79-268).  Without a GPU it exercises the argument checks and error paths; with one it
// also runs a filter, the device-resident loop, moments, a checkpoint / restore round trip (which
// must continue bitwise as the original) and the standalone resampler.  Exit status 0 = clean.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pf_engine.h"

static int fails = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c,     \
                   pf_last_error() ? pf_last_error() : "");                      \
      ++fails;                                                                   \
    }                                                                            \
  } while (0)

static pf_model_desc sv_model(std::vector<double>& A, std::vector<double>& beta, std::vector<double>& Q,
                              std::vector<double>& R, int nx) {
  A.assign((size_t)nx * nx, 0.0);
  for (int i = 0; i < nx; ++i) A[(size_t)i * nx + i] = 0.91;
  beta.assign(nx, 0.5);
  Q.assign((size_t)nx * nx, 0.0);
  R.assign((size_t)nx * nx, 0.0);
  for (int i = 0; i < nx; ++i) Q[(size_t)i * nx + i] = R[(size_t)i * nx + i] = 1.0;
  pf_model_desc m{};
  m.nx = nx;
  m.nz = nx;
  m.trans_kind = PF_TRANS_LINEAR;
  m.obs_kind = PF_OBS_EXP_HALF;
  m.trans_params = A.data();
  m.n_trans_params = (int64_t)A.size();
  m.obs_params = beta.data();
  m.n_obs_params = (int64_t)beta.size();
  m.Q = Q.data();
  m.R = R.data();
  return m;
}

static pf_opts opts_of(int64_t N, int R, int precision) {
  pf_opts o{};
  o.n_particles = N;
  o.n_replicates = R;
  o.resample_method = PF_RESAMPLE_SYSTEMATIC;
  o.resample_thresh = 0.5;
  o.precision = precision;
  o.seed = 42;
  return o;
}

static void error_paths() {
  CHECK(pf_version() != nullptr && std::strlen(pf_version()) > 0);
  std::vector<double> A, beta, Q, R;
  pf_model_desc m = sv_model(A, beta, Q, R, 1);
  pf_opts o = opts_of(1000, 1, PF_PRECISION_FP32);
  pf_handle* h = nullptr;
  CHECK(pf_create(nullptr, &o, &h) == PF_E_ARG && h == nullptr);
  CHECK(pf_create(&m, nullptr, &h) == PF_E_ARG && h == nullptr);
  CHECK(pf_create(&m, &o, nullptr) == PF_E_ARG);
  pf_model_desc bad = m;
  bad.nx = 0;
  CHECK(pf_create(&bad, &o, &h) != PF_OK && h == nullptr);
  bad = m;
  bad.n_trans_params = 0;  // A needs at least nx*nx values
  CHECK(pf_create(&bad, &o, &h) == PF_E_ARG && h == nullptr);
  bad = m;
  bad.n_obs_params = 0;  // beta needs at least nz values
  CHECK(pf_create(&bad, &o, &h) == PF_E_ARG && h == nullptr);
  pf_opts bo = o;
  bo.n_particles = 0;
  CHECK(pf_create(&m, &bo, &h) != PF_OK && h == nullptr);
  std::vector<double> Rn = {-1.0};  // not positive definite
  bad = m;
  bad.R = Rn.data();
  CHECK(pf_create(&bad, &o, &h) != PF_OK && h == nullptr);
  CHECK(pf_last_error() != nullptr);
  pf_destroy(nullptr);
  CHECK(pf_model_supported(1, 1, PF_TRANS_LINEAR, PF_OBS_EXP_HALF) == 1);
  CHECK(pf_model_supported(3, 1, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC) == 0);  // acoustic needs nx % 4 == 0
  CHECK(pf_model_supported(0, 1, PF_TRANS_LINEAR, PF_OBS_LINEAR) == 0);
  CHECK(pf_checkpoint_bytes(nullptr) < 0);
  CHECK(pf_run(nullptr, nullptr, nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr, nullptr) != PF_OK);
}

static void filter_run(int nx, int R, int precision) {
  std::vector<double> A, beta, Q, Rm;
  pf_model_desc m = sv_model(A, beta, Q, Rm, nx);
  const int64_t N = 1 << 16;
  pf_opts o = opts_of(N, R, precision);
  pf_handle* h = nullptr;
  CHECK(pf_create(&m, &o, &h) == PF_OK && h != nullptr);
  if (!h) return;
  std::vector<double> mean((size_t)R * nx, 0.0), cov((size_t)R * nx * nx, 0.0);
  for (int r = 0; r < R; ++r)
    for (int i = 0; i < nx; ++i) cov[((size_t)r * nx + i) * nx + i] = 1.0;
  CHECK(pf_initialize(h, mean.data(), cov.data(), nullptr) == PF_OK);
  const int64_t T = 64, T2 = 16;
  std::vector<double> Z((size_t)(T + T2) * R * nx);
  unsigned s = 7u;
  for (double& z : Z) {
    s = s * 1664525u + 1013904223u;
    z = 0.5 * std::exp(0.5 * (((s >> 8) & 0xffff) / 65536.0 - 0.5)) * (((s >> 24) & 1) ? 1.0 : -1.0);
  }
  std::vector<double> means((size_t)T * R * nx), neff((size_t)T * R), lnorm((size_t)T * R);
  std::vector<double> covs(nx <= 4 ? (size_t)T * R * nx * nx : 0);
  std::vector<uint8_t> flags((size_t)T * R);
  CHECK(pf_run(h, Z.data(), nullptr, T, 0, means.data(), covs.empty() ? nullptr : covs.data(), neff.data(),
               flags.data(), lnorm.data()) == PF_OK);
  for (double v : means) CHECK(std::isfinite(v));
  for (double v : neff) CHECK(v > 0.0 && v <= (double)N * 1.0000001);
  // checkpoint, continue, restore, continue again: the two continuations agree bitwise
  const int64_t nb = pf_checkpoint_bytes(h);
  CHECK(nb > 0);
  std::vector<unsigned char> blob((size_t)std::max<int64_t>(nb, 1));
  CHECK(pf_checkpoint(h, blob.data(), nb) == PF_OK);
  CHECK(pf_checkpoint(h, blob.data(), nb - 1) != PF_OK);  // short buffer refused
  std::vector<double> ma((size_t)T2 * R * nx), mb((size_t)T2 * R * nx);
  const double* Z2 = Z.data() + (size_t)T * R * nx;
  CHECK(pf_run(h, Z2, nullptr, T2, 0, ma.data(), nullptr, nullptr, nullptr, nullptr) == PF_OK);
  CHECK(pf_restore(h, blob.data(), nb) == PF_OK);
  CHECK(pf_run(h, Z2, nullptr, T2, 0, mb.data(), nullptr, nullptr, nullptr, nullptr) == PF_OK);
  CHECK(std::memcmp(ma.data(), mb.data(), ma.size() * sizeof(double)) == 0);
  // state readout and the exact two-pass moments
  std::vector<double> parts((size_t)R * N * nx), w((size_t)R * N), lw((size_t)R * N);
  CHECK(pf_get_particles(h, parts.data()) == PF_OK);
  CHECK(pf_get_weights(h, w.data(), lw.data()) == PF_OK);
  for (int r = 0; r < R; ++r) {
    double sw = 0.0;
    for (int64_t i = 0; i < N; ++i) sw += w[(size_t)r * N + i];
    CHECK(std::fabs(sw - 1.0) < 1e-6);
  }
  std::vector<double> m2((size_t)R * nx), c2((size_t)R * nx * nx);
  CHECK(pf_moments(h, m2.data(), c2.data()) == PF_OK);
  for (double v : m2) CHECK(std::isfinite(v));
  CHECK(pf_set_state(h, parts.data(), w.data()) == PF_OK);
  pf_destroy(h);
}

static void resampler() {
  const int64_t N = 10000;
  std::vector<double> w((size_t)N);
  for (int64_t i = 0; i < N; ++i) w[(size_t)i] = 1.0 / (double)N;
  std::vector<int64_t> idx((size_t)N, -1);
  CHECK(pf_resample_indices(0, PF_RESAMPLE_SYSTEMATIC, w.data(), N, 0.5, nullptr, idx.data()) == PF_OK);
  for (int64_t i = 0; i < N; ++i) CHECK(idx[(size_t)i] == i);  // equal weights: identity
}

int main() {
  error_paths();
  const int ndev = pf_device_count();
  std::printf("devices: %d\n", ndev);
  if (ndev > 0) {
    filter_run(1, 1, PF_PRECISION_FP32);
    filter_run(1, 4, PF_PRECISION_FP64);
    filter_run(4, 2, PF_PRECISION_FP32);
    resampler();
  }
  std::printf(fails ? "FAILED (%d)\n" : "ok\n", fails);
  return fails ? 1 : 0;
}
