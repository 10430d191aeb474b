"""NumPy restatement of the reference EDH particle-flow filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may
import this module; it is the checker for the HIP EDH flow, never the thing measured
or shipped.

Follows ``/root/reference/models/EDH_particle_filter.py`` (cited ``edh.py:LINE``):
``rk4_step`` 27-33, ``systematic_resample`` 35-47, ``effective_sample_size`` 49-52,
``EDHConfig`` 58-64, ``EDHFlowPF.init_from_gaussian`` 173-180, ``step`` 182-317,
``_weighted_stats`` 320-329.  The tracker, the plugin wirings and the weighted
statistics are shared with :mod:`oracle.ledh_oracle` (identical code in both reference
modules).  ``vectorized=True`` batches the per-particle RK4 of edh.py:273-275 (an
affine field, so the batched form is the same arithmetic per particle).
"""

from __future__ import annotations

import numpy as np

from oracle.ledh_oracle import LEDHModel, LEDHState, effective_sample_size, systematic_resample, weighted_stats

Array = np.ndarray


def rk4_step(x, f, dt):
    """edh.py:27-33."""
    k1 = f(x)
    k2 = f(x + 0.5 * dt * k1)
    k3 = f(x + 0.5 * dt * k2)
    k4 = f(x + dt * k3)
    return x + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)


class EDHOracle:
    """edh.py:149-329.  ``rng`` is the EDHConfig rng (edh.py:64)."""

    def __init__(self, tracker, model: LEDHModel, *, n_particles=512, n_lambda_steps=8, resample_ess_ratio=0.5,
                 flow_integrator="rk4", rng=None, vectorized=True):
        self.tracker = tracker
        self.m = model
        self.R = np.array(model.R, dtype=float)
        self.n_particles = int(n_particles)
        self.n_lambda_steps = int(n_lambda_steps)
        self.resample_ess_ratio = float(resample_ess_ratio)
        self.flow_integrator = flow_integrator
        self.rng = np.random.default_rng(0) if rng is None else rng
        self.vectorized = vectorized
        self.last_resampled = False
        self.last_ess = float("nan")

    def init_from_gaussian(self, mean0, cov0) -> LEDHState:
        """edh.py:173-180."""
        mean0 = np.asarray(mean0, float)
        eps = self.rng.multivariate_normal(np.zeros(mean0.size), cov0, size=self.n_particles)
        particles = mean0[None, :] + eps
        weights = np.full(self.n_particles, 1.0 / self.n_particles)
        mean, cov = weighted_stats(particles, weights)
        return LEDHState(particles, weights, mean, cov, {})

    def step(self, state: LEDHState, z_k, u_km1=None, process_noise_sampler=None) -> LEDHState:
        """edh.py:182-317."""
        m = self.m
        N, nx = state.particles.shape
        z_k = np.asarray(z_k, float)
        _, P = self.tracker.predict()
        P = 0.5 * (P + P.T)
        v = np.zeros((N, nx)) if process_noise_sampler is None else process_noise_sampler(N, nx)
        if self.vectorized:
            eta0 = m.g_vec(state.particles, u_km1, v)
        else:
            eta0 = np.empty_like(state.particles)
            for i in range(N):
                eta0[i] = m.g(state.particles[i], u_km1, v[i])
        eta = eta0.copy()
        etabar = m.g(self.tracker.get_past_mean(), u_km1, np.zeros(nx))
        n_steps = max(1, int(self.n_lambda_steps))
        dlam = 1.0 / float(n_steps)
        lam = 0.0
        I = np.eye(nx)
        cond_numbers = []
        for _ in range(n_steps):
            lam = min(1.0, lam + dlam)
            H = m.jac_h(etabar)
            h_bar = m.h(etabar)
            e = h_bar - H @ etabar
            S = lam * H @ P @ H.T + self.R
            try:
                cond_numbers.append(float(np.linalg.cond(S)))
            except Exception:
                cond_numbers.append(np.nan)
            try:
                S_inv_H = np.linalg.solve(S, H)
            except np.linalg.LinAlgError:
                S = S + 1e-8 * np.eye(S.shape[0])
                S_inv_H = np.linalg.solve(S, H)
            A = -0.5 * P @ H.T @ S_inv_H
            R_inv_innov = np.linalg.solve(self.R, (z_k - e))
            PHt_Rinv_innov = P @ H.T @ R_inv_innov
            b = (I + 2.0 * lam * A) @ ((I + lam * A) @ PHt_Rinv_innov + A @ etabar)

            def field(vec):
                return A @ vec + b

            if self.flow_integrator.lower() == "euler":
                eta = eta + dlam * (eta @ A.T + b)
                etabar = etabar + dlam * field(etabar)
            else:
                if self.vectorized:
                    eta = rk4_step(eta, lambda X: X @ A.T + b, dlam)
                else:
                    for i in range(N):
                        eta[i] = rk4_step(eta[i], field, dlam)
                etabar = rk4_step(etabar, field, dlam)
        xk = eta
        logw = np.log(state.weights + 1e-300)
        if self.vectorized:
            logw = logw + ((m.log_trans_vec(xk, state.particles) + m.log_like_vec(z_k, xk))
                           - m.log_trans_vec(eta0, state.particles))
        else:
            for i in range(N):
                logw[i] += (m.log_trans(xk[i], state.particles[i]) + m.log_like(z_k, xk[i])
                            - m.log_trans(eta0[i], state.particles[i]))
        logw -= np.max(logw)
        w = np.exp(logw)
        w /= np.sum(w)
        self.tracker.update(z_k)
        self.last_resampled = False
        self.last_ess = effective_sample_size(w)
        if self.resample_ess_ratio > 0.0:
            if self.last_ess < self.resample_ess_ratio * N:
                idx = systematic_resample(w, self.rng.random())
                xk = xk[idx]
                w = np.full_like(w, 1.0 / N)
                self.last_resampled = True
        mean, cov = weighted_stats(xk, w)
        return LEDHState(xk, w, mean, cov, {"condition_numbers": cond_numbers})


def run_edh(model: LEDHModel, Z, *, mean0, cov0, n_particles, n_lambda_steps, ratio, seed, integrator="rk4",
            noise=True, vectorized=True):
    """Drive the oracle like the reference tests (test_filters_mat_simulator.py:178-186)."""
    from oracle.ledh_oracle import make_ekf_tracker

    rng = np.random.default_rng(seed)
    tracker = make_ekf_tracker(model, mean0, cov0)
    pf = EDHOracle(tracker, model, n_particles=n_particles, n_lambda_steps=n_lambda_steps, resample_ess_ratio=ratio,
                   flow_integrator=integrator, rng=rng, vectorized=vectorized)
    st = pf.init_from_gaussian(mean0, cov0)
    init = st.particles.copy()
    T = len(Z)
    out = dict(means=np.zeros((T, model.nx)), covs=np.zeros((T, model.nx, model.nx)), ess=np.zeros(T),
               flags=np.zeros(T, dtype=bool), conds=np.zeros((T, max(1, n_lambda_steps))))
    sampler = (lambda N, nx: rng.multivariate_normal(np.zeros(nx), model.Q, size=N)) if noise else None
    for t in range(T):
        st = pf.step(st, np.atleast_1d(Z[t]), process_noise_sampler=sampler)
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["ess"][t] = pf.last_ess
        out["flags"][t] = pf.last_resampled
        out["conds"][t] = st.diagnostics["condition_numbers"]
    out["init_particles"] = init
    out["final_particles"] = st.particles.copy()
    out["final_weights"] = st.weights.copy()
    return out
