"""Paired multi-replicate free-run parity — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``tests/golden/make_golden_free_run.py`` and ``bench.py``'s parity leg may
use this module, as the checker.

The engine's native-Philox runs of the large-state configurations (BASELINE config 3, L96
d = 40; config 4, joint 16-D acoustic tracking) cannot be compared with the reference
trajectory by trajectory: fp32-vs-fp64 rounding flips a resample decision or an ancestor
within a few steps, after which the two filters are different Monte-Carlo draws of the same
algorithm.  SURVEY §8(c)(i) therefore asks for a statistical comparison: R >= 16 replicates
of the engine and of the fp64 oracle (:class:`oracle.sir_philox.PhiloxSIROracle`, the
reference algorithm of ``models/particle_filter.py:223-269`` on the engine's own Philox draws:
same seed, same replicate ids, same epochs), and the mean of the per-replicate paired
differences of each statistic within 3 standard errors of those differences, within a stated
relative equivalence margin (MARGINS), with the replicate count large enough that a bias of the
margin's size would be detected.

Statistics per replicate (over the scored window of steps):

* ``rmse``      sqrt(mean over steps and state dims of (posterior mean - truth)^2);
* ``loglik``    sum over steps of the log normaliser log sum_i w_{t-1,i} exp(-quad_i / 2)
                (the marginal-likelihood estimate up to the Gaussian constant; the weights'
                arithmetic, pf.py:256-262);
* ``resample_rate``  fraction of steps with Neff < 0.5 N (pf.py:203-204);
* ``omat``      (config 4) the MAT notebook's compute_omat per step (p = 1), averaged.

The oracle side is expensive (~1 s per L96 step at N = 1e5 in NumPy), so it is computed once
here in the build container and committed as numbers (tests/golden/free_run_pairs.npz, made by
tests/golden/make_golden_free_run.py); the engine side is run live on the GPU.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from . import omat_oracle
from .pf_oracle import run_filter
from .sir_philox import PhiloxSIROracle

# name -> replicates, particles, steps after initialize, first scored step (bench.py's warm-up W
# for config 4: the scored window is the bench's timed window [W, W + K))
CONFIGS = {
    "l96": dict(R=64, N=100_000, T=500, W=0, seed=42),  # config 3's full T = 500
    "mat": dict(R=512, N=100_000, T=110, W=10, seed=42, n_targets=4),
}
STATS = ("rmse", "loglik", "resample_rate", "omat")
# Stated equivalence margins: the largest relative bias |mean paired difference| / |oracle mean|
# the check accepts for each statistic.  The check also requires the power to see a bias of that
# size: its detectable bias 3 SE / |oracle mean| must not exceed the margin.  The margins are set
# from the oracle's own replicate spread at these replicate counts (sd / mean over replicates:
# L96 T = 500 RMSE 0.28 - runs that lose track of the 40-D state dominate it -, log-likelihood
# 0.39, resample rate 0.03; MAT RMSE 0.31, OMAT 0.32, log-likelihood 0.13, resample rate 0.05),
# i.e. they are the smallest biases these replicate counts can resolve, rounded up.
MARGINS = {
    "l96": {"rmse": 0.16, "loglik": 0.22, "resample_rate": 0.02},
    "mat": {"rmse": 0.065, "omat": 0.065, "loglik": 0.03, "resample_rate": 0.015},
}


def per_step(means, flags, lse, truth, n_targets: Optional[int] = None) -> Dict[str, np.ndarray]:
    """Per-step quantities of one replicate's run: squared error (mean over dims), flag, log
    normaliser and (n_targets given) the OMAT distance of the targets' positions."""
    means = np.asarray(means, float)
    truth = np.asarray(truth, float).reshape(means.shape)
    out = {"err2": np.mean((means - truth) ** 2, axis=1), "flags": np.asarray(flags, bool),
           "lse": np.asarray(lse, float)}
    if n_targets:
        T = means.shape[0]
        est = means.reshape(T, n_targets, -1)[:, :, :2]
        tru = truth.reshape(T, n_targets, -1)[:, :, :2]
        out["omat"] = np.array([omat_oracle.compute_omat(tru[t], est[t]) for t in range(T)])
    return out


def summarise(steps: Dict[str, np.ndarray], W: int) -> Dict[str, float]:
    """Per-replicate statistics over the scored window [W, T) of per_step() arrays."""
    s = {"rmse": float(np.sqrt(np.mean(steps["err2"][W:]))),
         "loglik": float(np.sum(steps["lse"][W:])),
         "resample_rate": float(np.mean(steps["flags"][W:]))}
    if "omat" in steps:
        s["omat"] = float(np.mean(steps["omat"][W:]))
    return s


def oracle_replicate(ssm, Z, truth, mean0, cov0, *, N, seed, rep, n_targets=None, bm24=True) -> dict:
    """The fp64 oracle on replicate ``rep``'s Philox draws (fresh handle: initialize at epoch 1,
    step t predicts at 2 + 2t), vectorised g/h; returns per_step() arrays."""
    o = PhiloxSIROracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, seed=seed, rep=rep, bm24=bm24, Np=N, vectorized=True,
                        c_normals=True)
    o.initialize(np.asarray(mean0, float).reshape(-1), np.asarray(cov0, float))
    r = run_filter(o, np.asarray(Z, float))
    return per_step(r["means"], r["flags"], r["lse"], truth, n_targets)


def paired_verdict(eng: Dict[str, np.ndarray], ora: Dict[str, np.ndarray], n_se: float = 3.0,
                   margins: Optional[Dict[str, float]] = None, name: Optional[str] = None) -> dict:
    """For each statistic (arrays over replicates, same replicate order on both sides): paired
    differences d_r = engine_r - oracle_r, their mean, standard error SE = sd(d)/sqrt(R), and
    three conditions, all required:

    * ``within_se``:   |mean| <= n_se * SE (no bias the replicates can resolve);
    * ``within_margin``: |mean| / |oracle mean| <= margin (MARGINS: the stated equivalence margin);
    * ``powered``:     the detectable bias n_se * SE / |oracle mean| <= margin, i.e. a bias as
      large as the margin would have failed ``within_se``.

    A statistic whose differences are all exactly zero passes trivially.  ``margins``: a statistic ->
    relative margin map, default MARGINS[name]."""
    if margins is None:
        if name not in MARGINS:
            raise ValueError("paired_verdict: give margins or a configuration name of MARGINS")
        margins = MARGINS[name]
    out = {}
    ok_all = True
    for k in STATS:
        if k not in eng or k not in ora:
            continue
        e, o = np.asarray(eng[k], float), np.asarray(ora[k], float)
        if e.shape != o.shape or e.ndim != 1 or e.size < 2:
            raise ValueError(f"paired_verdict: {k}: engine {e.shape} vs oracle {o.shape}")
        d = e - o
        R = d.size
        se = float(np.std(d, ddof=1) / np.sqrt(R))
        mean = float(np.mean(d))
        om = abs(float(np.mean(o)))
        margin = float(margins[k])
        exact = bool(np.all(d == 0))
        within_se = bool(abs(mean) <= n_se * se) or exact
        rel = abs(mean) / om if om > 0 else (0.0 if mean == 0 else np.inf)
        detectable = n_se * se / om if om > 0 else (0.0 if se == 0 else np.inf)
        within_margin = bool(rel <= margin)
        powered = bool(detectable <= margin) or exact
        ok = within_se and within_margin and powered
        ok_all &= ok
        out[k] = {"engine_mean": float(np.mean(e)), "oracle_mean": float(np.mean(o)),
                  "mean_paired_diff": mean, "se_paired_diff": se,
                  "z": mean / se if se > 0 else 0.0,
                  "relative_diff": float(rel), "detectable_bias_rel": float(detectable), "margin_rel": margin,
                  "within_se": within_se, "within_margin": within_margin, "powered": powered, "ok": ok,
                  # context: the replicates' own spread (independent Monte-Carlo draws)
                  "sd_engine": float(np.std(e, ddof=1)), "sd_oracle": float(np.std(o, ddof=1))}
    out["ok"] = ok_all
    out["n_se"] = n_se
    out["replicates"] = int(next(iter(eng.values())).shape[0]) if eng else 0
    return out
