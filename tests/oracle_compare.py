"""Engine-vs-oracle comparison on identical Philox draws (used by the -m gpu tests).

The fp32 engine and the fp64 oracle (oracle/sir_philox.c, the reference algorithm) consume
the same normals and uniforms.  Up to the first resample the only differences are fp32
arithmetic: SURVEY 8c's per-step tolerances (mean 1e-5 abs, Neff rel 1e-4) apply there (the
resample step itself excluded for the mean: its reported mean is the post-resample one).
At a resample, the fp32 state's rounding (~1e-7 relative per step, compounded through g)
moves ~0.1-1 % of the systematic positions (U + i) / N across an ancestor boundary; each
such slot takes an index neighbour - an unrelated particle - so from the first resample on
the two filters (even with the oracle forced to take the engine's decisions) differ at
Monte-Carlo level.  The yardstick there is the filter's own Monte-Carlo error, measured: the
same oracle run on an independent Philox seed.  The fp32-vs-fp64 per-step differences must
stay well inside it (RMS over the steps at most 0.75 of the independent-seed RMS; measured
0.41-0.56 at N = 3e5-1e6), and the free runs must meet the north-star |dRMSE| <= 1e-4 at
N = 1e6 (BASELINE.json).
"""

import numpy as np

from oracle import sir_philox as SP


def forced_compare(eng_means, eng_neff, eng_flags, model, Z, *, N, seed, mean0, var0, reg=False, bm24=True):
    flags = np.asarray(eng_flags, bool)
    o = SP.run_scalar(model, Z, N=N, seed=seed, mean0=mean0, var0=var0, bm24=bm24, regularize=reg,
                      forced=flags.astype(np.int32))
    indep = SP.run_scalar(model, Z, N=N, seed=seed + 7919, mean0=mean0, var0=var0, bm24=bm24, regularize=reg)
    own = o["neff"] < 0.5 * N
    disagree = np.nonzero(own != flags)[0]
    near = np.abs(o["neff"] - 0.5 * N) / N < 1e-3
    first = int(np.argmax(flags)) if flags.any() else len(flags)
    dmean = np.abs(np.asarray(eng_means, float) - o["means"])
    rel_neff = np.abs(np.asarray(eng_neff, float) / o["neff"] - 1.0)
    mc = np.abs(indep["means"] - o["means"])  # the filter's own Monte-Carlo error (independent seed)
    rms_d = float(np.sqrt(np.mean(dmean[first:] ** 2))) if first < len(flags) else 0.0
    rms_mc = float(np.sqrt(np.mean(mc[first:] ** 2))) if first < len(flags) else 1.0
    pre_mean = float(dmean[:first].max()) if first > 0 else 0.0
    return dict(first=first, dmean=dmean, rel_neff=rel_neff, disagree=disagree, pre_mean=pre_mean,
                rms_ratio=rms_d / rms_mc, near_ok=bool(np.all(near[disagree])), oracle=o,
                summary=(f"resamples {int(flags.sum())} (first at {first}); before it: max|dmean| {pre_mean:.2e}, "
                         f"max rel dNeff {rel_neff[:first + 1].max():.2e}; from it on: RMS dmean {rms_d:.2e} vs "
                         f"independent-seed RMS {rms_mc:.2e} (ratio {rms_d / rms_mc:.3f}), max|dmean| {dmean.max():.2e}, "
                         f"max rel dNeff {rel_neff.max():.2e}; oracle-vs-engine decisions differing {disagree.size}"))


def check_forced(c, *, tol_mean_pre=1e-5, tol_neff_pre=1e-4, tol_rms_ratio=0.75, tol_neff=5e-2):
    f = c["first"]
    assert c["near_ok"], f"decisions differ away from the threshold at {c['disagree']}"
    assert c["pre_mean"] <= tol_mean_pre
    assert c["rel_neff"][:f + 1].max() <= tol_neff_pre
    assert c["rms_ratio"] <= tol_rms_ratio
    assert c["rel_neff"].max() <= tol_neff
