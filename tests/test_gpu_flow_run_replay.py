"""The benchmarked LEDH / EDH device loop (``run()``: the fused one-launch step k_ledh_fused on the
linear-h path, the kernel chain otherwise) against the reference's own runs, head on (-m gpu).

tests/golden/ledh_runs.npz and edh_runs.npz hold the reference LEDHFlowPF / EDHFlowPF runs
(LEDH_particle_filter.py:93-214, EDH_particle_filter.py:182-317) with process noise and
resampling.  Their random stream is replayed into the device loop: after the initial draw,
step t's process_noise_sampler draw (rng.multivariate_normal(0, Q, N)) and - at the steps the
reference resampled - systematic_resample's rng.random() (ledh.py:28), laid out per step
(``run(..., process_noise="host", replay=(V, U))``, include/pf_ledh.h pf_ledh_set_run_replay).
The loop then takes its own decisions: they must equal the reference's.  Tolerances are those
of the step-API tests (tests/test_gpu_ledh.py, test_gpu_edh.py): every step's posterior mean
within 1e-9 x the state scale, covariance within 1e-8 x its scale, ESS rtol 1e-9 where no resample
reset it; the final particles within 1e-9 x scale and weights rtol 1e-7.
"""

import numpy as np
import pytest

from particle_filters_amd import _native as NV
from tests import test_gpu_edh as TE
from tests import test_gpu_ledh as TL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def replay_stream(cfg, Q, N, nx, flags):
    """The reference's draws after init_from_gaussian, in its order: noise every step, U on
    resample steps (NaN elsewhere: never read)."""
    T = len(flags)
    V = np.empty((T, N, nx))
    U = np.full(T, np.nan)
    for t in range(T):
        V[t] = cfg.rng.multivariate_normal(np.zeros(nx), Q, size=N)
        if flags[t]:
            U[t] = cfg.rng.random()
    return V, U


def check_run(pf, cfg, om, g, fused_expected=None):
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    np.testing.assert_array_equal(st.particles, g["init_particles"])
    N, nx = g["init_particles"].shape
    flags = np.asarray(g["flags"], bool)
    V, U = replay_stream(cfg, om.Q, N, nx, flags)
    res = pf.run(st, g["Z"], process_noise="host", replay=(V, U))
    assert np.array_equal(res.flags, flags), f"decisions {res.flags.astype(int)} vs reference {flags.astype(int)}"
    scale = max(1.0, float(np.abs(g["means"]).max()))
    np.testing.assert_allclose(res.means, g["means"], rtol=0, atol=1e-9 * scale)
    cs = np.maximum(1.0, np.abs(g["covs"]).max(axis=(1, 2)))[:, None, None]
    assert np.all(np.abs(res.covs - g["covs"]) <= 1e-8 * cs)
    fin = pf.state
    np.testing.assert_allclose(fin.particles, g["particles"][-1], rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(fin.weights, g["weights"][-1], rtol=1e-7, atol=1e-13)
    print(f"{g.get('name', '')}: T={len(flags)} N={N} resamples {int(flags.sum())}, max|dmean|/scale "
          f"{np.max(np.abs(res.means - g['means'])) / scale:.2e}")


@pytest.mark.parametrize("name", [n for n in TL.NAMES if n != "lin1d_nonoise"])
def test_ledh_run_replays_reference(name):
    pf, cfg, om, g = TL.make_filter(name)
    g = dict(g, name=f"LEDH {name} ({'fused step' if pf.shared_jacobian_path else 'kernel chain'})")
    check_run(pf, cfg, om, g)


@pytest.mark.parametrize("name", TE.NAMES)
def test_edh_run_replays_reference(name):
    pf, cfg, om, g = TE.make_filter(name)
    g = dict(g, name=f"EDH {name}")
    check_run(pf, cfg, om, g)
