"""The replicate-sharded multi-GPU path over RCCL (run on an MI355X: -m gpu).

SURVEY 8(e): independent Monte-Carlo replicates shard over ranks with one all-gather
of posterior summaries (``distributed.run_sharded``).  The CPU suite covers world
sizes 2-3 over gloo (tests/test_distributed.py); here the nccl (= RCCL) backend runs
for real, at world size 1 on the one GPU of the box, on BASELINE config 4's model
(joint 4-target acoustic tracking): the gathered summaries must equal a plain
``ParticleFilterBatch`` run bit for bit.
"""

import socket

import numpy as np
import pytest

from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_run_sharded_nccl_world1_matches_batch():
    import torch
    import torch.distributed as dist

    from particle_filters_amd.distributed import run_sharded

    assert NV.device_count() > 0
    cfg = S.ScenarioConfig(n_targets=4, n_steps=13, sensor_grid_shape=(5, 5), psi=10.0, d0=0.1, seed=56,
                           use_article_init=True)
    data = S.simulate_acoustic_dataset(cfg, S.DynamicsConfig())
    Q = np.kron(np.eye(4), S.article_process_noise_cov())
    R = 0.01 * np.eye(25)
    X = data["X"].reshape(13, 16)
    Z = data["Z"][1:]
    m0, c0 = X[0], np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0]))
    g, h = M.CVTransition(4, 1.0), M.AcousticObservation(data["S"], 10.0, 0.1, 4)
    kw = dict(Np=20000, seed=5, resample_thresh=0.5)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        res = run_sharded(g, h, Q, R, Z, mean0=m0, cov0=c0, n_replicates=3, device=0, **kw)
    finally:
        dist.destroy_process_group()
    b = ParticleFilterBatch(g, h, Q, R, n_replicates=3, **kw)
    b.initialize(m0, c0)
    ref = b.run(Z)
    b.close()
    assert ref.flags.sum() >= 1
    assert np.array_equal(res.means, ref.means)
    assert np.array_equal(res.covs, ref.covs)  # the device-loop covariance travels in the RCCL payload
    assert np.array_equal(res.neff, ref.neff)
    assert np.array_equal(res.flags, ref.flags)
    assert np.array_equal(res.log_norm, ref.log_norm)
