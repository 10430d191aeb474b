"""State-forced parity of EVERY step inside the benchmarked multi-step k_resident launch (-m gpu).

The register-resident kernel (csrc/pf_resident.h) runs all K steps of a run in one launch and
speculates past unverified steps; a resample found at verification rolls every workgroup back,
gathers, and recomputes the discarded steps.  tests/test_gpu_teacher_forced.py cuts runs into
one-step launches, which never speculate.  Here the launch the bench times is checked step by
step from the inside: while a trace is set (include/pf_engine.h pf_set_trace) the library runs
the trace instance of the same kernel, which stores, for every VERIFIED step (the version kept
after any rollback and recomputation), its predicted particles, its pre-resample log-weights and,
on a resample step, the ancestor of every output slot.  Each step t is then replayed by the fp64
oracle (oracle/sir_philox.c pfo_sir_scalar_check_step: pf.py:223-269 + _resample pf.py:188-220
on the engine's Philox draws) from the engine's own state before t - the traced state of step
t - 1, i.e. the previous step's predicted particles (resampled through the traced ancestors) and
weights - with identical draws.

Stated tolerances (fp32 engine; scale = max(1, E_w|x|) of the step; eps_w = the oracle-weighted
fp32 rounding bound of the engine's log-weights, computed per particle from the oracle's own
quantities - 2^-21 (1 + |l| + |log-likelihood|) + the fp32 observation and the predicted particle's
rounding through the likelihood's slopes (sir_philox.c) - a formula, not a measured engine error):
  predicted particles     |dx| <= 2e-6 x scale
  weights                 total variation <= min(max(1e-7, eps_w), 1e-3)
  Neff                    rel <= min(max(1e-5, 4 eps_w), 4e-3)
  decision                identical unless Neff is within 1e-3 N of 0.5 N
  ancestors               every slot holds a valid, non-decreasing ancestor; where it differs from
                          searchsorted over the engine's own weights (fp64 cumsum of its fp32
                          log-weights) the slot's position lies within band_self = 2^-20 (1 +
                          E_w|l - max l|) of that ancestor's interval (the fp32 exponentials and
                          tile sums of the engine's CDF); where it differs from the oracle's
                          ancestor, within band_self + 2 eps_w (|dcdf| <= 2 TV)
  posterior mean          <= 1e-5 x scale against the oracle's set under the engine's decision
                          and ancestors
  posterior variance      <= (2e-5 + 4 dx / sigma) x max(var, (1e-6 scale)^2)
  chained state           after the launch, the engine's state is exactly the traced chain's
                          (particles bitwise; weights rel 8 x 2^-24 (1 + max|l|): the exit log-weights
                          are the last traced ones shifted by <= 3 verified frame deltas in fp32)
Every measured quantity and its bound per step goes to $PF_EVIDENCE_DIR (default
gpurun_out/evidence) as JSON; the round's copy is kept under profiles/.
"""

import json
import os
import time

import numpy as np
import pytest

from tests import teacher_forced as TF

import bench
from oracle import sir_philox as SP
from particle_filters_amd import _native as NV
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu

TOL_X = 2e-6
TOL_MEAN = 1e-5
TOL_COV = 2e-5
BAND_SELF_ULP = 2.0 ** -20


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _evidence(name, payload):
    d = os.environ.get("PF_EVIDENCE_DIR", os.path.join("gpurun_out", "evidence"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w") as f:
        json.dump(payload, f, indent=1)


def _softmax(l):
    l = np.asarray(l, float)
    m = np.max(l)
    w = np.exp(l - m)
    return w / w.sum()


class TraceChain:
    """Replays the traced steps of the runs of one SV filter through the C oracle."""

    def __init__(self, T_cap, n_particles=None):
        self.wl = bench.WORKLOADS["sv"]()
        self.N = int(n_particles or self.wl.n_particles)
        self.model = SP.sv_logsq_model(bench.ALPHA, bench.SIGMA, bench.BETA)
        self.lib = NV.load()
        self.T_cap = T_cap
        self.records = []
        self.worst = {}

    def make(self, T_data):
        g, h, Q, R, Z, truth, mean0, cov0 = self.wl.build(T_data, 0)
        self.Z = np.asarray(Z, float).reshape(T_data, -1)
        pf = ParticleFilterBatch(g, h, Q, R, Np=self.N, n_replicates=1, seed=42)
        pf.initialize(mean0, cov0)
        return pf, mean0, cov0

    def run(self, pf, a, b, label):
        """Run Z[a:b] as ONE resident launch with the trace on and check every step of it."""
        NV.check(self.lib.pf_set_trace(pf.handle, b - a), "pf_set_trace")
        x = pf.particles()[0, :, 0].copy()
        w = pf.weights()[0].copy()
        ep0 = int(pf.rng_state()["epoch"])
        res = pf.run(self.Z[a:b])
        assert pf.last_run_resident, "the run did not take the register-resident kernel"
        N = self.N
        xe = np.empty(N, np.float32)
        le = np.empty(N, np.float32)
        anc = np.empty(N, np.int32)
        prev_res = [False, False]
        for t in range(b - a):
            NV.check(self.lib.pf_get_trace(pf.handle, t, 0, NV.C.c_void_p(xe.ctypes.data),
                                           NV.C.c_void_p(le.ctypes.data), NV.C.c_void_p(anc.ctypes.data)),
                     "pf_get_trace")
            flag = bool(res.flags[t, 0])
            c = SP.check_step(self.model, seed=42, rep=0, epoch=ep0 + 2 * t, thresh=0.5, x0=x, w0=w, z=self.Z[a + t],
                              xe=xe, le=le, anc=anc if flag else None, neff_e=res.neff[t, 0], flag_e=flag,
                              mean_e=res.means[t, 0, 0], var_e=res.covs[t, 0, 0, 0])
            if not flag:
                assert np.all(anc == -1), "ancestors traced on a step that did not resample"
            we = _softmax(le)
            c.update(self._bounds(c, le, we))
            c["t"] = a + t
            c["launch"] = label
            c["step_in_launch"] = t
            c["recomputed_after_rollback"] = bool(prev_res[0] or prev_res[1])
            self._check(c)
            self.records.append({k: (float(v) if isinstance(v, (np.floating, float)) else v) for k, v in c.items()})
            prev_res = [flag, prev_res[0]]
            # the engine's state after step t: the traced predicted particles, resampled through the
            # traced ancestors, with uniform weights - or its weights as they are
            if flag:
                x = xe[anc].astype(float)
                w = np.full(N, 1.0 / N)
            else:
                x = xe.astype(float)
                w = we
        # the chained state IS the engine's state after the launch: particles bitwise; the exit
        # log-weights are the last traced ones shifted by the frame deltas of the steps verified after
        # it (at most LAG + 1 = 3), each rounded to fp32: rel <= 8 x 2^-24 (1 + max |l|)
        xf, wf = pf.particles()[0, :, 0], pf.weights()[0]
        assert np.array_equal(xf, x), f"{label}: exit particles differ from the traced chain"
        lmax = 0.0 if flag else float(np.max(np.abs(le[np.isfinite(le)])))
        np.testing.assert_allclose(wf, w, rtol=8.0 * 2.0 ** -24 * (1.0 + lmax), atol=1e-12 / N)
        NV.check(self.lib.pf_set_trace(pf.handle, 0), "pf_set_trace")
        return res

    @staticmethod
    def _bounds(c, le, we):
        scale = max(1.0, c["mean_abs_x"])
        fin = np.isfinite(le)
        spread = float(np.sum(we[fin] * (np.max(le[fin]) - le[fin].astype(float))))
        band_self = BAND_SELF_ULP * (1.0 + spread)
        sigma = float(np.sqrt(max(c["var_o"], (1e-6 * scale) ** 2)))
        # the rounding bound, capped by the fixed ceilings of tests/teacher_forced.py (TV 1e-3, Neff 4e-3)
        return dict(scale=scale, tv_bound=min(max(1e-7, c["eps_w"]), TF.TV_CEILING),
                    neff_bound=min(max(1e-5, 4.0 * c["eps_w"]), TF.NEFF_CEILING),
                    band_self=band_self, band_oracle=band_self + 2.0 * c["eps_w"],
                    var_rel=c["dvar"] / max(c["var_o"], (1e-6 * scale) ** 2),
                    var_bound=TOL_COV + 4.0 * c["dx_pre"] / sigma)

    def _check(self, c):
        s = c["scale"]
        ratios = {"dx_pre": c["dx_pre"] / (TOL_X * s), "tv_w": c["tv_w"] / c["tv_bound"],
                  "neff_rel": c["neff_rel"] / c["neff_bound"], "dmean": c["dmean"] / (TOL_MEAN * s),
                  "var": c["var_rel"] / c["var_bound"],
                  "margin_self": c["max_margin_self"] / c["band_self"],
                  "margin_oracle": c["max_margin_oracle"] / c["band_oracle"]}
        for k, v in ratios.items():
            if v > self.worst.get(k, (-1.0, None))[0]:
                self.worst[k] = (float(v), int(c["t"]))
        msg = json.dumps({k: c[k] for k in ("t", "launch", "flag_e", "flag_o", "dx_pre", "tv_w", "tv_bound", "neff_rel",
                                            "n_anc_bad", "n_anc_self_diff", "max_margin_self", "band_self",
                                            "n_anc_oracle_diff", "max_margin_oracle", "band_oracle", "dmean",
                                            "var_rel", "var_bound")})
        assert ratios["dx_pre"] <= 1.0, msg
        assert ratios["tv_w"] <= 1.0, msg
        assert ratios["neff_rel"] <= 1.0, msg
        if c["flag_e"] != c["flag_o"]:
            assert c["near_threshold"], msg
        assert c["n_anc_bad"] == 0, msg
        assert ratios["margin_self"] <= 1.0, msg
        assert ratios["margin_oracle"] <= 1.0, msg
        assert ratios["dmean"] <= 1.0, msg
        assert ratios["var"] <= 1.0, msg

    def summary(self):
        r = self.records
        res = [x for x in r if x["flag_e"]]
        return {"steps_checked": len(r), "resample_steps": len(res),
                "recomputed_steps_checked": sum(x["recomputed_after_rollback"] for x in r),
                "decision_flips_near_threshold": sum(x["flag_e"] != x["flag_o"] for x in r),
                "anc_self_diff_slots_total": int(sum(x["n_anc_self_diff"] for x in res)),
                "anc_oracle_diff_slots_total": int(sum(x["n_anc_oracle_diff"] for x in res)),
                "worst_ratio_to_bound": {k: {"ratio": v[0], "step": v[1]} for k, v in self.worst.items()}}


def test_trace_instance_equals_shipped_kernel():
    """The trace instance computes exactly what the shipped instance computes (same outputs
    bitwise over a 20-step launch with a resample): only stores were added."""
    tc = TraceChain(40)
    pf1, _, _ = tc.make(45)
    pf2, _, _ = tc.make(45)
    NV.check(tc.lib.pf_set_trace(pf2.handle, 40), "pf_set_trace")
    r1, r2 = pf1.run(tc.Z[:40]), pf2.run(tc.Z[:40])
    assert pf1.last_run_resident and pf2.last_run_resident
    assert r1.flags.sum() >= 1
    for a, b in ((r1.means, r2.means), (r1.neff, r2.neff), (r1.covs, r2.covs), (r1.log_norm, r2.log_norm)):
        assert np.array_equal(a, b)
    assert np.array_equal(r1.flags, r2.flags)
    assert np.array_equal(pf1.particles(), pf2.particles())
    pf1.close()
    pf2.close()


def test_resident_trace_driver_window():
    """The driver's bench window at BASELINE config 2 (N = 1e6): bench.py's default is initialize,
    a 5-step warm-up launch, then ONE timed 20-step launch that contains a resample (rollback,
    hand-off, 2 recomputed steps).  Every step of both launches is checked."""
    tc = TraceChain(20)
    pf, _, _ = tc.make(25)
    t0 = time.time()
    tc.run(pf, 0, 5, "warmup_K5")
    r = tc.run(pf, 5, 25, "timed_K20")
    pf.close()
    s = tc.summary()
    s["seconds"] = time.time() - t0
    _evidence("resident_trace_driver_window.json", {"summary": s, "steps": tc.records})
    print(json.dumps(s))
    assert r.flags.sum() >= 1, "no resample inside the timed window"
    assert s["recomputed_steps_checked"] >= 1


def test_resident_trace_config2_k1000():
    """BASELINE config 2 as one 1000-step launch (N = 1e6, T = 1000, seed 42): all 1000 in-launch
    steps, ~55 resamples with their rollbacks and recomputed steps."""
    tc = TraceChain(1000)
    pf, _, _ = tc.make(1000)
    t0 = time.time()
    r = tc.run(pf, 0, 1000, "K1000")
    pf.close()
    s = tc.summary()
    s["seconds"] = time.time() - t0
    _evidence("resident_trace_k1000.json", {"summary": s, "steps": tc.records})
    print(json.dumps(s))
    assert r.flags.sum() >= 20
