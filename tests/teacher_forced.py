"""State-teacher-forced one-step parity of the benchmarked fp32 kernels (helper of the -m gpu tests).

At a step boundary t of a benchmarked run the engine's own fp32 state S_t (particles, normalised
log-weights, Philox position: ``ParticleFilterBatch.checkpoint`` / ``rng_state``) is loaded into
the fp64 oracle (``oracle.sir_philox.PhiloxSIROracle`` = ``oracle.pf_oracle.SIROracle``, pinned bit
for bit to the reference's outputs, on the engine's Philox draws) and both run ONE step
(pf.py:223-269 + _resample pf.py:188-220) with identical draws.  The comparison is split so each
part has a sharp tolerance:

1. the pre-resample step.  The engine's predicted particles and weights come from a twin handle
   with resample_thresh = 0 into which the same checkpoint is restored (the same kernel, the same
   arithmetic; only the decision differs): particles within fp32 rounding, the weights' total
   variation distance, Neff (rel), the decision (it may differ only where Neff is within 1e-3 N of
   the threshold);
2. the engine's resampling on its own weights: the post-step particles are EXACTLY
   ``x'_e[searchsorted(cumsum(w_e), (U + i)/N, 'right')]`` (+ the jitter), U the step's Philox
   uniform - bit-exact indices, except where a position lies within 1e-12 of the engine's CDF
   (fp64 summation order);
3. the engine's ancestors against the oracle's: they differ only at near-ties, i.e. slots whose
   position lies within band = 2 eps_w + 2^-22 of the oracle's CDF interval of the engine's ancestor
   (|cdf_e - cdf_o| <= 2 TV <= 2 eps_w, plus the engine's fp32 exponentials), and the posterior mean
   equals the oracle's with the engine's ancestors within 1e-5 x scale.

eps_w is the fp32 rounding bound of the engine's log-weights, weighted by the oracle's weights and
computed per particle from the ORACLE's quantities only (never from a measured engine-oracle
difference): rnd (1 + |log w0| + |log-likelihood| + sum_j |(R^-1 (z - h))_j| (|h_j| + |z_j|)) - rnd = 8
unit roundoffs (2^-21 for fp32) over the carried log-weight's shift, the likelihood's operations and
the fp32 observation / predictions it is built from - plus the change of the oracle's likelihood
under any particle perturbation within part 1's tolerance, tol_x x scale x |J_h^T R^-1 (z - h)|_1
(the oracle's likelihood gradient, ``ll_rounding_bound``).  The weights' total variation must stay
within max(tol_tv, eps_w), Neff within max(tol_neff, 4 eps_w).
"""

from __future__ import annotations

import numpy as np

from oracle import sir_philox as SP
from oracle.pf_oracle import OracleState, systematic_indices


class StepOracle(SP.PhiloxSIROracle):
    """PhiloxSIROracle that keeps the pre-resample particles / weights and the systematic U."""

    def _resample(self, particles, weights):
        self.pre_x = np.array(particles, float)
        self.pre_w = np.array(weights, float)
        self.U = None
        self.idx = None
        return super()._resample(particles, weights)

    def _systematic_resample(self, weights):
        self.U = float(self.rng.random())
        self.idx = systematic_indices(weights, self.U)
        return self.idx


def margins(w, U, idx):
    """|position - nearest edge of the chosen ancestor's CDF interval| per slot (fp64 cumsum)."""
    N = len(w)
    cdf = np.cumsum(w)
    cdf[-1] = 1.0
    pos = (U + np.arange(N)) / N
    lo = np.where(idx > 0, cdf[np.maximum(idx - 1, 0)], 0.0)
    return np.minimum(pos - lo, cdf[idx] - pos), cdf, pos


def ll_rounding_bound(h_vec, X, gz, dx, hjt_vec=None):
    """Per particle, a bound on |ll(x + d) - ll(x)| over the perturbations |d_k| <= dx_k, from the
    ORACLE's particles: ll = 1/2 |LR^-1 (z - h(x))|^2 has the gradient -J_h(x)^T R^-1 (z - h(x)) =
    -J_h^T gz, so |dll| <= sum_k dx_k |J_h^T gz|_k to first order; the gradient from the model's
    analytic J_h^T (ssm.hjt_vec) or by central differences of phi(x) = gz . h(x) (gz held fixed), and
    a factor 1.25 for the second-order term (dx is a few fp32 ulps of the state).  dx: a scalar (the
    same box for every component) or [N][nx] (each particle's own deviation)."""
    X = np.asarray(X, float)
    N, nx = X.shape
    dx = np.broadcast_to(np.asarray(dx, float), (N, nx))
    if hjt_vec is not None:
        return 1.25 * np.sum(np.abs(np.asarray(hjt_vec(X, np.asarray(gz, float).T), float)) * dx, axis=1)
    g1 = np.zeros(N)
    for k in range(nx):
        d = 1e-6 * np.maximum(1.0, np.abs(X[:, k]))
        xp, xm = X.copy(), X.copy()
        xp[:, k] += d
        xm[:, k] -= d
        hp = np.asarray(h_vec(xp), float).reshape(N, -1)
        hm = np.asarray(h_vec(xm), float).reshape(N, -1)
        g1 += np.abs(np.sum((hp - hm).T * gz, axis=0) / (2.0 * d)) * dx[:, k]
    return 1.25 * g1


def one_step(ssm, Q, R, *, seed, rep, epoch, thresh, method, reg, x0, w0, z, xe_pre, we_pre, neff_e, neff_e0,
             flag_e, mean_e, xe_post, scale, bm24=True, rnd=2.0 ** -21, exp_err=2.0 ** -22, K=8, cov_e=None,
             cov_floor=1e-6, tol_x=2e-6):
    """Compare one engine step with the oracle's from the same state.  Returns a dict of measured
    quantities (see module docstring); tolerances are applied by ``check``."""
    N, nx = x0.shape
    o = StepOracle(ssm.g_vec, ssm.h_vec, Q, R, seed=seed, rep=rep, bm24=bm24, epoch=epoch, Np=N,
                   resample_thresh=thresh, resample_method=method, regularize_after_resample=reg, vectorized=True)
    o.state = OracleState(np.array(x0, float), np.array(w0, float), np.zeros(nx), np.eye(nx), 0)
    st = o.step(np.atleast_1d(np.asarray(z, float)))
    out = dict(N=N)
    # 1. pre-resample: particles, weights, Neff, decision
    out["dx_pre"] = float(np.max(np.abs(xe_pre - o.pre_x)))
    out["tv_w"] = float(0.5 * np.sum(np.abs(we_pre - o.pre_w)))
    cdf_o = np.cumsum(o.pre_w)
    cdf_e = np.cumsum(we_pre)
    out["dcdf"] = float(np.max(np.abs(cdf_e - cdf_o)))
    out["neff_rel"] = float(abs(neff_e / o.last_neff - 1.0))
    # the fp32 rounding the weights carry: 2^-24 x the log-likelihood magnitude per particle (a few
    # ulps of |l| - large for MAT's 25 sensors at R = 0.01 I), weighted by the posterior
    zz = np.atleast_1d(np.asarray(z, float))
    hx = np.asarray(ssm.h_vec(o.pre_x), float).reshape(N, -1)
    resid = np.linalg.solve(o.LR, (zz - hx).T)  # [nz][N]
    ll = 0.5 * np.sum(resid * resid, axis=0)
    out["lmag"] = float(np.sum(o.pre_w * ll))
    # the fp32 rounding bound of the engine's log-weights (module docstring), oracle quantities only
    gz = np.linalg.solve(o.LR.T, resid)  # R^-1 (z - h), [nz][N]
    hz = np.sum(np.abs(gz) * (np.abs(hx.T) + np.abs(zz)[:, None]), axis=0)
    # the particle-rounding term: each particle's own state deviation |x'_e - x'_o| (part 1 checks
    # it is within tol_x x scale) through the likelihood's slope; eps_w_box keeps the whole-box
    # version (every component at tol_x x scale) for reference
    hjt = getattr(ssm, "hjt_vec", None)
    dll = ll_rounding_bound(ssm.h_vec, o.pre_x, gz, np.abs(np.asarray(xe_pre, float) - o.pre_x), hjt)
    dll_box = ll_rounding_bound(ssm.h_vec, o.pre_x, gz, tol_x * scale, hjt)
    with np.errstate(divide="ignore"):
        lw0 = np.abs(np.log(np.asarray(w0, float) + 1e-300))
    base = rnd * (1.0 + lw0 + ll + hz)
    out["eps_w"] = float(np.sum(o.pre_w * (base + dll)))
    out["eps_w_box"] = float(np.sum(o.pre_w * (base + dll_box)))
    out["neff_twin_equal"] = bool(neff_e == neff_e0)
    out["flag_e"], out["flag_o"] = bool(flag_e), bool(o.last_resampled)
    out["near_threshold"] = bool(abs(o.last_neff - thresh * N) / N < 1e-3)
    out["resampled"] = bool(flag_e)
    out["dcov"] = out["dcov_self"] = 0.0
    out["sigma"] = 1.0
    if not flag_e:
        out["dx_post"] = float(np.max(np.abs(xe_post - xe_pre)))  # no resample: the state is x'_e itself
        mo = st.mean if not o.last_resampled else np.average(o.pre_x, axis=0, weights=o.pre_w)
        out["dmean"] = float(np.max(np.abs(mean_e - mo)))
        if cov_e is not None:  # pf.py:266-267 on the weighted predicted particles
            co = np.atleast_2d(np.cov(o.pre_x.T, aweights=o.pre_w, bias=True))
            cs = np.atleast_2d(np.cov(xe_pre.T, aweights=we_pre, bias=True))  # the engine's own set
            den = max(np.max(np.abs(co)), (cov_floor * scale) ** 2)
            out["dcov"] = float(np.max(np.abs(cov_e - co)) / den)
            out["dcov_self"] = float(np.max(np.abs(cov_e - cs)) / den)
            out["sigma"] = float(np.sqrt(max(np.max(np.diag(co)), (cov_floor * scale) ** 2)))
        out["dmean_oracle"] = out["dmean"]
        out["n_anc_self_mismatch"] = out["n_anc_diff"] = 0
        out["max_margin_diff"] = 0.0
        return out
    assert method == "systematic"
    # the step's systematic U and jitter normals (the oracle's own draws, whatever it decided)
    U = float(SP.philox.uniform53(seed, 0, rep, epoch + 1))
    jit = np.zeros_like(xe_post)
    if reg:  # 0.001 chol(Q) n on the resample epoch's jitter stream (pf.py:212-218)
        try:
            Lq = np.linalg.cholesky(Q)
        except np.linalg.LinAlgError:
            Lq = np.linalg.cholesky(Q + 1e-12 * np.eye(nx))
        jit = o.prng.at(epoch + 1, SP.philox.STREAM_JITTER).standard_normal((N, nx)) @ (0.001 * Lq.T)
    # 2. the engine's ancestors, read off its post-step particles: slot i holds x'_e[j] (+ the slot's
    #    jitter) for one j; candidates are the oracle's ancestor and its index neighbours
    idx_o = systematic_indices(o.pre_w, U)
    if o.idx is not None:
        assert np.array_equal(idx_o, o.idx)
    cdf_o = np.cumsum(o.pre_w)
    cdf_o[-1] = 1.0
    pos = (U + np.arange(N)) / N
    band = 2.0 * out["eps_w"] + exp_err  # |cdf_e - cdf_o| <= 2 TV <= 2 eps_w, plus the engine's exponentials

    def dist(j):  # distance of pos to the oracle's CDF interval of ancestor j
        lo = np.where(j > 0, cdf_o[np.maximum(j - 1, 0)], 0.0)
        return np.maximum(0.0, np.maximum(lo - pos, pos - cdf_o[j]))

    tol_copy = 0.0 if not reg else 4e-7 * scale  # a copy is exact (the jitter: fp32 vs fp64 add)
    idx_e = np.full(N, -1, dtype=np.int64)
    for k in sorted(range(-K, K + 1), key=abs):
        cand = np.clip(idx_o + k, 0, N - 1)
        todo = idx_e < 0
        if not todo.any():
            break
        hit = np.max(np.abs(xe_post[todo] - (xe_pre[cand[todo]] + jit[todo])), axis=1) <= tol_copy
        sel = np.nonzero(todo)[0][hit]
        idx_e[sel] = cand[sel]
    # a near-tie may also skip particles of (numerically) zero weight, far away in index: the slots
    # not matched near the oracle's ancestor are looked up among all predicted particles (exact
    # row lookup; with jitter, a scan of at most 256 slots)
    rest = np.nonzero(idx_e < 0)[0]
    if rest.size and not reg:
        rows = {}
        for j, key in enumerate(map(bytes, np.ascontiguousarray(xe_pre))):
            rows.setdefault(key, []).append(j)
        for i in rest:
            m = np.asarray(rows.get(bytes(np.ascontiguousarray(xe_post[i])), []), dtype=np.int64)
            if m.size:  # the copy whose oracle CDF interval is nearest the slot's position
                lo = np.where(m > 0, cdf_o[np.maximum(m - 1, 0)], 0.0)
                idx_e[i] = m[np.argmin(np.maximum(0.0, np.maximum(lo - pos[i], pos[i] - cdf_o[m])))]
    elif 0 < rest.size <= 256:
        for i in rest:
            m = np.nonzero(np.max(np.abs(xe_pre + jit[i] - xe_post[i]), axis=1) <= tol_copy)[0]
            if m.size:
                lo = np.where(m > 0, cdf_o[np.maximum(m - 1, 0)], 0.0)
                idx_e[i] = m[np.argmin(np.maximum(0.0, np.maximum(lo - pos[i], pos[i] - cdf_o[m])))]
    out["n_unmatched"] = int(np.sum(idx_e < 0))
    diff = (idx_e >= 0) & (idx_e != idx_o)
    d = dist(np.maximum(idx_e, 0))
    out["n_anc_diff"] = int(np.sum(diff))
    out["max_margin_diff"] = float(np.max(d[diff])) if diff.any() else 0.0
    out["band"] = band
    idx_e = np.where(idx_e >= 0, idx_e, idx_o)
    forced = o.pre_x[idx_e] + jit
    out["dmean"] = float(np.max(np.abs(mean_e - forced.mean(axis=0))))
    out["dmean_oracle"] = float(np.max(np.abs(mean_e - st.mean)))
    out["dx_post"] = float(np.max(np.abs(xe_post - forced)))
    out["n_anc_self_mismatch"] = out["n_unmatched"]
    if cov_e is not None:  # pf.py:266-267 on the resampled set (uniform weights), the engine's ancestors
        co = np.atleast_2d(np.cov(forced.T, bias=True))
        # relative to the covariance, or to (cov_floor x state scale)^2 for a (near-)degenerate set
        # (a resampled set of copies: np.cov gives O(1e-32), the engine exactly 0 or O(eps^2 |x|^2))
        den = max(np.max(np.abs(co)), (cov_floor * scale) ** 2)
        out["dcov"] = float(np.max(np.abs(cov_e - co)) / den)
        cs = np.atleast_2d(np.cov(xe_post.T, bias=True))  # the engine's own post-resample set
        out["dcov_self"] = float(np.max(np.abs(cov_e - cs)) / den)
        out["sigma"] = float(np.sqrt(max(np.max(np.diag(co)), (cov_floor * scale) ** 2)))
    return out


# Fixed ceilings on the weight tolerances (advisor, round 5): whatever the rounding bound says, the
# total variation of the weights may not exceed 1e-3 and Neff may not move by more than 4e-3.
TV_CEILING, NEFF_CEILING = 1e-3, 4e-3


def bounds(c, *, scale, tol_x=2e-6, tol_mean=1e-5, tol_neff=1e-5, tol_tv=1e-7):
    """The step's stated bounds (see ``check``)."""
    return dict(x=tol_x * scale, tv=min(max(tol_tv, c["eps_w"]), TV_CEILING),
                neff=min(max(tol_neff, 4.0 * c["eps_w"]), NEFF_CEILING),
                mean=tol_mean * scale, band=c.get("band", 0.0))


def check(c, *, scale, tol_x=2e-6, tol_mean=1e-5, tol_neff=1e-5, tol_tv=1e-7, tol_cov=2e-5):
    """Tolerances (stated in the test module): particles tol_x x scale (fp32 rounding of one step),
    weights' TV distance max(tol_tv, eps_w) and Neff rel max(tol_neff, 4 eps_w), eps_w the rounding
    bound of the module docstring, capped at TV_CEILING = 1e-3 and NEFF_CEILING = 4e-3; decisions identical unless Neff is within 1e-3 N of the
    threshold; every post-step slot is a copy of one of the engine's predicted particles whose
    oracle CDF interval lies within band = 2 eps_w + 2^-22 of the position; the posterior mean
    within tol_mean x scale of the oracle's particles under the engine's ancestors; the covariance
    within tol_cov of np.cov of the engine's own set, and of the oracle's set within tol_cov + 4 dx / sigma."""
    b = bounds(c, scale=scale, tol_x=tol_x, tol_mean=tol_mean, tol_neff=tol_neff, tol_tv=tol_tv)
    assert c["neff_twin_equal"], "the twin (thresh 0) step must have the same Neff bit for bit"
    assert c["dx_pre"] <= b["x"], c
    assert c["tv_w"] <= b["tv"], c
    assert c["neff_rel"] <= b["neff"], c
    if c["flag_e"] != c["flag_o"]:
        assert c["near_threshold"], c
    assert c["n_anc_self_mismatch"] == 0, c
    if c["resampled"]:
        assert c["max_margin_diff"] <= c["band"], c
    assert c["dmean"] <= tol_mean * scale, c
    # the covariance of the engine's own set to tol_cov; against the oracle's set, plus the first-order
    # effect of the particles' fp32 rounding (dC / C ~ 2 dx / sigma)
    assert c["dcov_self"] <= tol_cov, c
    assert c["dcov"] <= tol_cov + 4.0 * c["dx_pre"] / c["sigma"], c
    assert c["dx_post"] <= 2 * tol_x * scale, c


def fmt(t, c):
    return (f"t={t:4d} res={int(c['flag_e'])}/{int(c['flag_o'])} dx_pre={c['dx_pre']:.2e} tvw={c['tv_w']:.2e} "
            f"eps_w={c['eps_w']:.2e} "
            f"dcdf={c['dcdf']:.2e} dNeff={c['neff_rel']:.2e} dmean={c['dmean']:.2e} (vs oracle's own "
            f"ancestors {c['dmean_oracle']:.2e}) anc_diff={c['n_anc_diff']} max_margin={c['max_margin_diff']:.2e} "
            f"band={c.get('band', 0.0):.2e} unmatched={c['n_anc_self_mismatch']} dcov/|cov| self {c['dcov_self']:.2e} "
            f"oracle {c['dcov']:.2e}")
