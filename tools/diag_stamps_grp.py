"""Per-phase timing of k_step_grp (MAT / L96) from s_memrealtime stamps (PF_STAMPS build).
usage: PF_LIB=build/libpf_hip_stamps.so python tools/diag_stamps_grp.py mat|l96"""
import os, sys
import ctypes as C
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch
lib = NV.load()
wl = sys.argv[1] if len(sys.argv) > 1 else "mat"
fn = getattr(lib, "pf_debug_stamps_" + wl)
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
if wl == "mat":
    cfg = S.ScenarioConfig(n_targets=4, n_steps=60, sensor_grid_shape=(5, 5), seed=56)
    d = S.simulate_acoustic_dataset(cfg, S.DynamicsConfig())
    pf = ParticleFilterBatch(M.CVTransition(4, 1.0), M.AcousticObservation(d["S"], 10.0, 0.1, 4),
                             np.kron(np.eye(4), S.article_process_noise_cov()), 0.01 * np.eye(25), Np=100000,
                             n_replicates=8, seed=1)
    pf.initialize(d["X"][0].ravel(), np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0])))
    Z = d["Z"][1:]
else:
    sim = S.simulate_lorenz96(nx=40, spinup_steps=1000, total_steps=60, Np=1, obs_interval=1, obs_fraction=4, seed=42)
    pf = ParticleFilterBatch(M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40), 0.01 * np.eye(40),
                             sim.R, Np=100000, seed=1)
    pf.initialize(sim.ensemble_traj[0, 0], 2.0 * np.eye(40))
    Z = sim.observations[1:]
G, tile, lds = pf.geometry()
SL = 10
for T in (20, 40, 59):
    res = pf.run(Z[:T])
    n = min(G, 4096)
    buf = (C.c_ulonglong * (n * SL))()
    assert fn(buf, n * SL) == 0
    a = np.array(buf[:], dtype=np.float64).reshape(n, SL)[:, :6]
    rel = (a - a[:, 0].min()) / 100.0
    print(f"{wl} T={T} G={G} tile={tile} last flag={res.flags[-1].tolist()}")
    for k, nm in enumerate(["entry", "prologue", "outputs", "ancestors", "chunks", "record"]):
        col = rel[:, k]
        print(f"  {nm:10s} min {col.min():8.2f} med {np.median(col):8.2f} max {col.max():8.2f} us")
