"""Engine-vs-oracle comparison on identical Philox draws (used by the -m gpu tests).

The fp32 engine and the fp64 oracle (oracle/sir_philox.c, the reference algorithm) consume
the same normals and uniforms.  Up to the first resample the only differences are fp32
arithmetic: SURVEY 8c's per-step tolerances (mean 1e-5 abs, Neff rel 1e-4) apply there.  At
a resample, the fp32 state's rounding (~1e-7 relative per step, compounded through g) moves
~0.1-1 % of the systematic positions (U + i) / N across an ancestor boundary; each such
slot takes an index neighbour - an unrelated particle - so from the first resample on, the
two filters (even with the oracle forced to take the engine's decisions) differ at Monte-
Carlo level.  Those steps are held to a fraction of the filter's own Monte-Carlo standard
error of the posterior mean, sqrt(var_t / Neff_t), and the free runs to the north-star
|dRMSE| <= 1e-4 at N = 1e6 (BASELINE.json).
"""

import numpy as np

from oracle import sir_philox as SP


def forced_compare(eng_means, eng_neff, eng_flags, model, Z, *, N, seed, mean0, var0, reg=False, bm24=True):
    flags = np.asarray(eng_flags, bool)
    o = SP.run_scalar(model, Z, N=N, seed=seed, mean0=mean0, var0=var0, bm24=bm24, regularize=reg,
                      forced=flags.astype(np.int32))
    own = o["neff"] < 0.5 * N
    disagree = np.nonzero(own != flags)[0]
    near = np.abs(o["neff"] - 0.5 * N) / N < 1e-3
    first = int(np.argmax(flags)) if flags.any() else len(flags)
    dmean = np.abs(np.asarray(eng_means, float) - o["means"])
    rel_neff = np.abs(np.asarray(eng_neff, float) / o["neff"] - 1.0)
    se = np.sqrt(np.maximum(o["vars"], 0.0) / o["neff"])
    ratio = dmean / se
    return dict(first=first, dmean=dmean, rel_neff=rel_neff, ratio=ratio, disagree=disagree,
                near_ok=bool(np.all(near[disagree])), oracle=o,
                summary=(f"resamples {int(flags.sum())} (first at {first}); up to it: max|dmean| "
                         f"{dmean[:first + 1].max():.2e}, max rel dNeff {rel_neff[:first + 1].max():.2e}; all steps: "
                         f"max|dmean| {dmean.max():.2e} (median {np.median(dmean):.1e}), max |dmean|/SE "
                         f"{ratio.max():.2f} (99% {np.quantile(ratio, 0.99):.2f}), max rel dNeff {rel_neff.max():.2e}; "
                         f"oracle-vs-engine decisions differing {disagree.size}"))


def check_forced(c, *, tol_mean_pre=1e-5, tol_neff_pre=1e-4, tol_ratio=1.0, tol_neff=5e-2):
    f = c["first"]
    assert c["near_ok"], f"decisions differ away from the threshold at {c['disagree']}"
    assert c["dmean"][:f + 1].max() <= tol_mean_pre
    assert c["rel_neff"][:f + 1].max() <= tol_neff_pre
    assert c["ratio"].max() <= tol_ratio
    assert c["rel_neff"].max() <= tol_neff
