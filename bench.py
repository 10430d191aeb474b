#!/usr/bin/env python
"""Benchmark: BASELINE config 2 — SIR filter on the 1-D SV model, N = 1e6 particles.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload sv|l96|mat]

One *step* = one filter time step (predict + weight + ESS + resample-if-needed +
posterior summary) over all particles of every replicate a GPU holds.  Each rank
(one process per GPU, ``torch.distributed`` over RCCL when N > 1) runs its own
independent Monte-Carlo replicates (Philox replicate ids = its global block) on
the same synthetic series; per-GPU work is fixed ("weak" scaling).  The timed
region is W-step warm-up excluded, then exactly K steps of the device-resident
loop (``pf_run_device``: inputs already in HBM, no host sync inside), followed by
the RCCL all-gather of every replicate's posterior summaries (means, ESS, flags),
bracketed by barrier + device synchronisation; the max over ranks is reported.

Workloads (BASELINE.json configs; the default is the headline metric's config):
  sv   config 2: 1-D SV log-squared wiring, N = 1e6, one replicate per GPU
  l96  config 3: Lorenz-96 d = 40 (RK4 g, every 4th component observed), N = 1e5
  mat  config 4: joint 4-target acoustic tracking (nx = 16, nz = 25), N = 1e5,
       8 replicates per GPU (64 over 8 GPUs)
  ledh config 5: LEDH particle flow on L96 d = 40, N = 1e4, 8 lambda steps (fp64)
  edh  config 5's job with the EDH global flow (EDH_particle_filter.py, RK4) (fp64)
  ledh_mat  the MAT notebook's joint LEDH run: 16-D, 25 sensors, N = 500, L = 64, 39 steps (fp64)

Extra JSON fields:
  roofline      dominant kernel.  SV: k_resident<f32, SV> — ONE launch runs all K
                steps with the particles register-resident (pf_resident.h).
                L96/MAT: k_step (one launch per step).  achieved = algorithmic
                bytes (N x (8 nx + 8) per replicate-step, + N x
                (8 nx + 12) on resample steps) of the timed run / its device
                duration, timed live with HIP events recorded on the engine's own
                stream; traffic = HBM bytes per step from the committed rocprofv3
                PMC passes (profiles/pmc_traffic*.json), or null; valu = the
                kernel's VALU issue floor per step (profiles/pmc_valu_*.json,
                SQ_INSTS_VALU) and the fraction of the measured step it covers.
  cpu_baseline  the reference CPU path (faithful per-particle restatement in
                oracle/, bit-identical to the reference) timed on this host's cores
                on a bounded sample of the same workload.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "particle-steps/sec (N×T/s) + RMSE vs CPU ref, SV model N=1e6"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ALPHA, SIGMA, BETA = 0.95, 0.2, 1.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(workload, kernel):
    """HBM bytes per filter step of `kernel` from the committed PMC summary, if present."""
    name = "pmc_traffic.json" if workload == "sv" else f"pmc_traffic_{workload}.json"
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        d = json.load(fh)
    if d.get("kernel_short") != kernel:
        return None, None
    return d.get("bytes_per_step"), d.get("source")


def pmc_valu(workload, kernel, us_per_step):
    """VALU issue floor of `kernel` per filter step from the committed PMC summary
    (tools/pmc_valu.py: SQ_INSTS_VALU x 2 cycles / occupied SIMDs / 2.4 GHz), if present."""
    path = os.path.join(REPO, "profiles", f"pmc_valu_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    if d.get("kernel_short") != kernel:
        return None
    fl = d["issue_floor_us_per_step"]
    return {"valu_insts_per_step": d["valu_insts_per_step"], "issue_floor_us_per_step": fl,
            "frac": fl / us_per_step, "simds": d["simds"], "source": d["source"]}


class Workload:
    """Inputs, filter construction and CPU baseline of one BASELINE config."""

    name = ""
    n_particles = 0
    replicates = 1
    nx = nz = 1
    kernel_tmpl = ""
    defaults = (1000, 100)  # steps, warmup

    def build(self, T, rank):  # -> (g, h, Q, R, Z [T][nz], truth [T][nx], mean0, cov0)
        raise NotImplementedError

    def oracle_ssm(self):
        raise NotImplementedError

    def describe(self, world):
        raise NotImplementedError


class SV(Workload):
    name, n_particles, replicates, nx, nz = "sv", 1_000_000, 1, 1, 1
    kernel_tmpl = "float,1,1,LINEAR,LINEAR"
    cpu_steps = 6

    def build(self, T, rank):
        from particle_filters_amd import models as M, simulators as S

        data = S.simulate_sv_1d(T + 1, ALPHA, SIGMA, BETA, seed=42)
        Z = np.log(data.Y[1:] ** 2)[:, None]  # log-squared wiring (PF_VS_experiments.ipynb cell 6)
        self.X0 = data.X[0]
        return (M.SVTransition(ALPHA), M.SVLogSqObservation(BETA), [[SIGMA ** 2]], [[M.LOGCHI2_VAR]], Z,
                data.X[1:, None], [data.X[0]], [[0.5]])

    def oracle_ssm(self):
        from oracle import ssm_oracle

        return ssm_oracle.sv_logsq(ALPHA, SIGMA, BETA)

    def describe(self, world):
        return ("SIR bootstrap PF, 1-D SV (BASELINE config 2): N=1e6 particles per GPU, "
                "systematic resampling at Neff<0.5N, T=steps",
                "synthetic (simulate_sv_1d alpha=0.95 sigma=0.2 beta=1 seed=42, log-squared wiring)")


class SV64(SV):
    """SURVEY 8(d) roofline run for C2: 64 independent SV filters of N=1e6 each per GPU (Philox
    replicate ids stand for the per-replicate seeds 42+r); the 1 GB working set exceeds the
    256 MB MALL, so the launch-per-step kernel streams the state through HBM."""

    name, replicates = "sv64", 64
    defaults = (100, 10)
    cpu_steps = 6

    def describe(self, world):
        return (f"SIR bootstrap PF, 1-D SV (BASELINE config 2 roofline run, SURVEY 8d): {self.replicates} "
                f"independent filters x N=1e6 particles per GPU ({self.replicates * world} total), systematic "
                "resampling at Neff<0.5N, T=steps",
                "synthetic (simulate_sv_1d alpha=0.95 sigma=0.2 beta=1 seed=42, log-squared wiring; "
                "one observation sequence, Philox replicate ids per filter)")


class L96(Workload):
    name, n_particles, replicates, nx, nz = "l96", 100_000, 1, 40, 10
    kernel_tmpl = "float,40,10,L96,LINEAR"
    defaults = (500, 50)
    cpu_steps = 2

    def build(self, T, rank):
        from particle_filters_amd import models as M, simulators as S

        sim = S.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=T, Np=1,
                                  obs_interval=1, obs_fraction=4, obs_error_std=1.0, seed=42)
        Q = 0.1 ** 2 * np.eye(40)  # the build's choice (truth is noise-free, simulator_Lorenz_96.py:394)
        return (M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40), Q, sim.R,
                sim.observations[1:], sim.truth_traj[1:], sim.ensemble_traj[0, 0], 2.0 * np.eye(40))

    def oracle_ssm(self):
        from oracle import ssm_oracle

        return ssm_oracle.lorenz96(nx=40, q_std=0.1)

    def describe(self, world):
        return ("SIR bootstrap PF, Lorenz-96 d=40 (BASELINE config 3): RK4 dt=0.01 F=8, every 4th component "
                "observed (R=I), Q=0.01 I, N=1e5 particles per GPU, systematic resampling at Neff<0.5N",
                "synthetic (simulate_lorenz96 nx=40 spinup=1000 obs_interval=1 obs_fraction=4 seed=42)")


class MAT(Workload):
    name, n_particles, replicates, nx, nz = "mat", 100_000, 8, 16, 25
    kernel_tmpl = "float,16,25,LINEAR,ACOUSTIC"
    defaults = (100, 10)
    cpu_steps = 2

    def build(self, T, rank):
        from particle_filters_amd import models as M, simulators as S

        cfg = S.ScenarioConfig(n_targets=4, n_steps=T + 1, sensor_grid_shape=(5, 5), psi=10.0, d0=0.1, seed=56,
                               use_article_init=True)
        data = S.simulate_acoustic_dataset(cfg, S.DynamicsConfig())
        self.S = data["S"]
        Qs = S.article_process_noise_cov()
        Q = np.kron(np.eye(4), Qs)
        R = 0.01 * np.eye(25)
        X = data["X"].reshape(T + 1, 16)
        return (M.CVTransition(4, 1.0), M.AcousticObservation(data["S"], 10.0, 0.1, 4), Q, R, data["Z"][1:],
                X[1:], X[0], np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0])))

    def oracle_ssm(self):
        from oracle import ssm_oracle

        return ssm_oracle.mat_joint(self.S)

    def describe(self, world):
        return (f"SIR bootstrap PF, joint 4-target acoustic tracking (BASELINE config 4): nx=16, 5x5 sensors, "
                f"N=1e5 particles x {self.replicates} replicates per GPU ({self.replicates * world} total), "
                "systematic resampling at Neff<0.5N",
                "synthetic (simulate_acoustic_dataset 4 targets seed=56 article init, R=0.01 I)")


class L96Big(L96):
    """simulate_lorenz96's default dimension (nx = 1000, every 4th component observed): outside
    the compiled shape list, so it runs on the runtime-shape kernels (csrc/pf_dyn.h)."""

    name, n_particles, replicates, nx, nz = "l96_1000", 16_384, 1, 1000, 250
    kernel_tmpl = "float,L96,LINEAR"
    defaults = (50, 5)
    cpu_steps = 1

    def build(self, T, rank):
        from particle_filters_amd import models as M, simulators as S

        sim = S.simulate_lorenz96(nx=1000, F=8.0, dt=0.01, spinup_steps=1000, total_steps=T, Np=1,
                                  obs_interval=1, obs_fraction=4, obs_error_std=1.0, seed=42)
        Q = 0.1 ** 2 * np.eye(1000)
        return (M.L96Transition(8.0, 0.01, 1000), M.SelectObservation(sim.H_idx, 1000), Q, sim.R,
                sim.observations[1:], sim.truth_traj[1:], sim.ensemble_traj[0, 0], 2.0 * np.eye(1000))

    def oracle_ssm(self):
        from oracle import ssm_oracle

        return ssm_oracle.lorenz96(nx=1000, q_std=0.1)

    def describe(self, world):
        return ("SIR bootstrap PF, Lorenz-96 d=1000 (simulate_lorenz96's default size; runtime-shape kernels): "
                "RK4 dt=0.01 F=8, every 4th component observed (R=I), Q=0.01 I, N=16384 particles per GPU, "
                "systematic resampling at Neff<0.5N",
                "synthetic (simulate_lorenz96 nx=1000 spinup=1000 obs_interval=1 obs_fraction=4 seed=42)")


WORKLOADS = {"sv": SV, "sv64": SV64, "l96": L96, "l96_1000": L96Big, "mat": MAT, "ledh": None, "edh": None,
             "ledh_mat": None}
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec (half the FP32 vector 157.3 TF of MI355X_MICROARCH.md)


def ledh_flops_per_particle(nx, nz, L):
    """Algorithmic FP64 flops of one particle-step of the shared-Jacobian LEDH flow
    (pf_ledh_kernels.h k_flow_shared): RK4 g (4 rhs x 4 nx + 3 stage axpys x 2 nx + final
    3 nx), chol(Q) noise (nx(nx+1)/2 FMA), y0 = H eta0 (nx nz FMA), per lambda step
    2 nz^2 + nx nz FMA + ~4 nz + 3 nx, two diagonal quadratic forms (2 nx) + one nz^2."""
    rk4 = 4 * 4 * nx + 3 * 2 * nx * 2 + 3 * nx
    noise = nx * (nx + 1)  # FMA = 2 flops
    y0 = 2 * nx * nz
    per_lam = 2 * (2 * nz * nz + nx * nz) + 4 * nz + 3 * nx
    quad = 2 * 2 * nx + 2 * nz * nz
    return rk4 + noise + y0 + L * per_lam + quad


def ledh_pp_flops_per_particle(nx, nz, L):
    """Algorithmic FP64 flops of one particle-step of the per-particle LEDH flow in the
    reference's formulation (LEDH_particle_filter.py:136-179): per lambda step P H^T
    (2 nx^2 nz), S = lam H P H^T + R (2 nz^2 nx), its factorisation and the solve for
    S^-1 H ((2/3) nz^3 + 2 nz^2 nx), A = -1/2 P H^T S^-1 H (2 nx^2 nz), b and the
    eta update (~10 nx^2), slogdet(I + dlam A) ((2/3) nx^3)."""
    per_lam = 4 * nx * nx * nz + 4 * nz * nz * nx + (2 * nz ** 3) // 3 + (2 * nx ** 3) // 3 + 10 * nx * nx
    return L * per_lam


def main_ledh(args, world, rank, local, algo="ledh", use_dist=False, model="l96"):
    """BASELINE config 5: LEDH particle flow on Lorenz-96 d = 40, N = 1e4, 8 lambda steps
    (algo="edh": the same job with the EDH global flow of EDH_particle_filter.py, RK4 integrator).
    model="mat": the reference's one published LEDH run — joint 4-target acoustic tracking
    (16-D state, 25 sensors), N = 500, 64 lambda steps, 39 filter steps over the 40-step
    scenario, 2095.74 s in the reference notebook
    (PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb:1095, cells 5-6)."""
    import torch

    torch.cuda.set_device(local)
    dist = None
    if use_dist:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from particle_filters_amd import edh as ED, ledh as LD, models as M, simulators as S, trackers as TR

    if model == "mat":
        K = args.steps if args.steps is not None else 39
        W = args.warmup if args.warmup is not None else 3
        Np, L, nx, nz = 500, 64, 16, 25
        cfg_s = S.ScenarioConfig(n_targets=4, n_steps=max(40, W + K + 1), sensor_grid_shape=(5, 5), psi=10.0, d0=0.1,
                                 seed=56, use_article_init=True)
        data = S.simulate_acoustic_dataset(cfg_s, S.DynamicsConfig())
        g, h = M.CVTransition(4, 1.0), M.AcousticObservation(data["S"], 10.0, 0.1, 4)
        Q, R = np.kron(np.eye(4), S.article_process_noise_cov()), 0.1 ** 2 * np.eye(25)
        Xt = data["X"].reshape(data["X"].shape[0], 16)
        # the notebook's joint prior: per-target N(mean, diag(10^2, 10^2, 1, 1)) around the start
        mean0 = Xt[0] + np.tile([1.5, -1.0, 0.1, -0.1], 4)
        cov0 = np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0]))
        Zs, truth_all = data["Z"], Xt
    else:
        K = args.steps if args.steps is not None else 200
        W = args.warmup if args.warmup is not None else 20
        Np, L, nx, nz = 10_000, 8, 40, 10
        sim = S.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=W + K, Np=1, obs_interval=1,
                                  obs_fraction=4, obs_error_std=1.0, seed=42)
        g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40)
        Q, R = 0.1 ** 2 * np.eye(40), sim.R
        mean0, cov0 = sim.ensemble_traj[0, 0], 2.0 * np.eye(40)
        Zs, truth_all = sim.observations, sim.truth_traj

    def make():
        ekf = TR.ExtendedKalmanFilter(g, h, Q, R, jac_g=g.jacobian, jac_h=h.jacobian)
        tracker = TR.EKFTracker(ekf, TR.EKFState(mean0.copy(), cov0.copy(), 0))
        args_ = (tracker, g, h, h.jacobian, M.GaussianTransitionDensity(g, Q), M.GaussianLikelihood(h, R), R)
        if algo == "edh":
            cfg = ED.EDHConfig(n_particles=Np, n_lambda_steps=L, resample_ess_ratio=0.5, flow_integrator="rk4",
                               rng=np.random.default_rng(42 + rank))
            return ED.EDHFlowPF(*args_, cfg, rng_mode="device"), tracker
        cfg = LD.LEDHConfig(n_particles=Np, n_lambda_steps=L, resample_ess_ratio=0.5,
                            rng=np.random.default_rng(42 + rank))
        return LD.LEDHFlowPF(*args_, cfg, rng_mode="device"), tracker

    Z = Zs[1:]
    pf, tracker = make()
    st = pf.init_from_gaussian(mean0, cov0)
    pf.run(st, Z[:max(W, 1)], tracker="device")  # warm-up (same sequence as the timed run)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    # the whole job on the device: EKF tracker (k_ekf_seq), all flow tables, then the T flow steps
    res = pf.run(pf.state, Z[W:W + K], tracker="device")
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0  # before the closing barrier (max over ranks below)
    if dist:
        dist.barrier()
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # host-tracker variant (the reference's call pattern: tracker stepped in Python), for the record
    pf2, tracker2 = make()
    st2 = pf2.init_from_gaussian(mean0, cov0)
    pf2.run(st2, Z[:max(W, 1)])
    h0 = time.perf_counter()
    Ps = np.empty((K, nx, nx))
    Xb = np.empty((K, nx))
    for t in range(K):
        _, P = tracker2.predict()
        Ps[t] = P
        Xb[t] = tracker2.get_past_mean()
        tracker2.update(Z[W + t])
    t_tr = time.perf_counter() - h0
    if algo == "edh":
        pf2.run(pf2.state, Z[W:W + K], tracker_seq=(Ps, Xb))
    else:
        pf2.run(pf2.state, Z[W:W + K], tracker_covs=Ps)
    torch.cuda.synchronize()
    t_host_total = time.perf_counter() - h0
    pf2.close()
    dev_s = elapsed
    rmse = res.rmse(truth_all[W + 1:W + K + 1])
    per_particle = pf.shared_jacobian_path is False
    fpp = ledh_pp_flops_per_particle(nx, nz, L) if per_particle else ledh_flops_per_particle(nx, nz, L)
    flops = fpp * Np * K
    if model == "mat":
        wl_name = "joint 4-target acoustic tracking (16-D state, 25 sensors)"
        data_desc = ("synthetic (simulate_acoustic_dataset 4 targets 5x5 sensors psi=10 d0=0.1 seed=56 article init; "
                     "R=0.01 I, Q=blockdiag(article_process_noise_cov))")
        notes = (f"N={Np} particles, {L} lambda steps, ESS-ratio 0.5 systematic resampling, EKF tracker on the device "
                 "(analytic acoustic Jacobian), per-particle LEDH flow in the targets' position space "
                 "(pf_ledh_kernels.h k_flow_wave_lr), Philox noise")
    else:
        wl_name = "L96 d=40"
        data_desc = "synthetic (simulate_lorenz96 nx=40 spinup=1000 obs_interval=1 obs_fraction=4 seed=42)"
        notes = ("N=1e4 particles, 8 lambda steps, ESS-ratio 0.5 systematic resampling, EKF tracker on the device "
                 "(analytic RK4 Jacobian), Philox process noise")
    # the per-particle flow kernel: the position-space one for the acoustic h with diagonal R
    flow_kernel = ("k_flow_wave_lr" if model == "mat" else "k_flow_wave") if per_particle else "k_ledh_fused"
    ltraffic = pmc_traffic("ledh_mat" if (model == "mat" and algo == "ledh") else algo, flow_kernel)[0]
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            from oracle import edh_oracle as EO, ledh_oracle as LO

            if model == "mat":
                om = LO.acoustic_joint(h.S, psi=10.0, d0=0.1, n_targets=4, Q_single=S.article_process_noise_cov())
                n_cpu = 100
            else:
                om = LO.lorenz96(40)
                n_cpu = 1000
            steps = int(os.environ.get("PF_CPU_BASELINE_STEPS", "1"))
            tr = LO.make_ekf_tracker(om, mean0, cov0)
            if algo == "edh":
                opf = EO.EDHOracle(tr, om, n_particles=n_cpu, n_lambda_steps=L, resample_ess_ratio=0.5,
                                   rng=np.random.default_rng(1), vectorized=False)
            else:
                opf = LO.LEDHOracle(tr, om, n_particles=n_cpu, n_lambda_steps=L, resample_ess_ratio=0.5,
                                    rng=np.random.default_rng(1), vectorized=False)
            ost = opf.init_from_gaussian(mean0, cov0)
            sampler = lambda n, d: opf.rng.multivariate_normal(np.zeros(d), om.Q, size=n)  # noqa: E731
            c0 = time.perf_counter()
            for t in range(steps):
                ost = opf.step(ost, Z[t], process_noise_sampler=sampler)
            cdt = time.perf_counter() - c0
            cpu = {"value": n_cpu * steps / cdt, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                   "sample": f"{algo.upper()} {wl_name}, N={n_cpu}, L={L}, {steps} step(s), faithful per-particle "
                             f"restatement (oracle/{algo}_oracle.py, bit-identical to the reference "
                             f"{algo.upper()}FlowPF), {cdt:.1f} s",
                   "cores_on_host": os.cpu_count()}
        # The roofline of the per-particle flow (the acoustic LEDH run): the kernel's executed VALU
        # issue rate against the issue peak of the SIMDs it occupies (profiles/pmc_valu_ledh_mat.json:
        # SQ_INSTS_VALU per step, 2 cycles per wave instruction at 2.4 GHz), not the reference
        # formulation's dense flop count, which the position-space kernel does not execute.
        vinfo = pmc_valu("ledh_mat" if (model == "mat" and algo == "ledh") else algo, flow_kernel, dev_s * 1e6 / K)
        if per_particle and vinfo is not None:
            issue_peak = vinfo["simds"] * 2400.0 / 2.0  # wave instructions per us
            issued = vinfo["valu_insts_per_step"] / (dev_s * 1e6 / K)
            roof = {"bound": "fp64-valu-issue", "achieved": issued, "peak": issue_peak,
                    "unit": "VALU wave-instructions/us", "frac": issued / issue_peak,
                    "reference_formulation_tflops": flops / dev_s / 1e12,
                    "reference_formulation_frac_of_fp64_peak": flops / dev_s / 1e12 / FP64_VALU_PEAK_TFLOPS}
        else:
            roof = {"bound": "fp64-valu", "achieved": flops / dev_s / 1e12, "peak": FP64_VALU_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": flops / dev_s / 1e12 / FP64_VALU_PEAK_TFLOPS}
        line = {
            "metric": f"particle-steps/sec (N×T/s), {algo.upper()} flow filter {wl_name}",
            "value": Np * K * world / elapsed, "unit": "particle-steps/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": elapsed * 1e3 / K, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64",
            "data": data_desc,
            "config": {"workload": (("LEDH particle-flow PF" + (" (BASELINE config 5)" if model == "l96" else
                                                                  " (the MAT notebook's joint LEDH run)"))
                                    if algo == "ledh" else
                                    "EDH particle-flow PF (the global EDH flow, RK4)") + f": {wl_name}, " + notes,
                       "n_particles": Np, "n_lambda": L, "shared_jacobian_path": pf.shared_jacobian_path,
                       "parallelism": f"replicas x{world} (one independent filter per GPU)"},
            "rmse": rmse, "resample_rate": float(np.mean(res.flags)),
            "host_tracker_variant": {"ms_per_step": t_host_total * 1e3 / K, "tracker_ms_per_step": t_tr * 1e3 / K,
                                     "note": "EKF stepped on the host in NumPy, covariances uploaded, same device loop"},
            "roofline": {**roof,
                         "traffic": ltraffic,
                         "traffic_gbs": None if ltraffic is None else ltraffic / (dev_s / K) / 1e9,
                         "traffic_frac": None if ltraffic is None else ltraffic / (dev_s / K) / 1e9 / HBM_PEAK_GBS,
                         "traffic_unit": "HBM bytes per filter step of the kernel (rocprofv3 FETCH_SIZE x2 + "
                                         "WRITE_SIZE, profiles/pmc_traffic_<workload>.json)",
                         "kernel": ("whole LEDH job: k_ekf_seq + " + (f"per step {flow_kernel} (per-particle flow)"
                                                                      if per_particle else
                                                                      "k_setup/k_compose + per step k_ledh_fused"))
                                   if algo == "ledh" else "whole EDH job: k_ekf_seq + k_edh_setup + per step k_ledh_fused",
                         "flops_per_particle_step": fpp,
                         "flops_note": "the reference formulation's per-particle dense algebra (estimate; the "
                                       "position-space kernel executes far fewer: frac is its VALU issue rate)"
                                       if per_particle else "shared-Jacobian flow (see ledh_flops_per_particle)",
                         "valu": vinfo},
            "cpu_baseline": cpu,
        }
        if model == "mat" and algo == "ledh":
            ref_s = 2095.74  # PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb:1095 (N=500, 39 steps)
            line["reference_published"] = {
                "value": 500 * 39 / ref_s, "unit": "particle-steps/s", "seconds": ref_s,
                "source": "PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb:1095 (joint LEDH, N=500, "
                          "L=64, 39 steps; reference NumPy on the authors' machine)",
                "speedup": (Np * K * world / elapsed) / (500 * 39 / ref_s)}
        print(json.dumps(line), flush=True)
    pf.close()
    if dist:
        dist.destroy_process_group()


def cpu_baseline(wl, Z, mean0, cov0):
    """Faithful reference CPU path (per-particle Python g/h, particle_filter.py:237,257)
    on a bounded sample: the bench workload (one replicate) for a few steps, 1 core."""
    from oracle import pf_oracle

    steps = min(int(os.environ.get("PF_CPU_BASELINE_STEPS", str(wl.cpu_steps))), len(Z))
    ssm = wl.oracle_ssm()
    pf = pf_oracle.SIROracle(ssm.g, ssm.h, ssm.Q, ssm.R, Np=wl.n_particles, rng=np.random.default_rng(42))
    pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
    t0 = time.perf_counter()
    for t in range(steps):
        pf.step(Z[t])
    dt = time.perf_counter() - t0
    return {"value": wl.n_particles * steps / dt, "unit": "particle-steps/s", "cores": 1, "kind": "port",
            "sample": f"{wl.name} N={wl.n_particles:.0e}, 1 replicate, {steps} steps, faithful per-particle "
                      f"restatement (oracle/pf_oracle.py, bit-identical to the reference), {dt:.1f} s"}


def cpu_baseline_numpy(wl, Z, mean0, cov0):
    """SURVEY.md 8(d) CPU variant (2): the same restatement with vectorised NumPy g/h
    (one array op per step instead of N Python calls), 1 core, on a bounded sample."""
    from oracle import pf_oracle

    steps = min(int(os.environ.get("PF_CPU_NUMPY_STEPS", str(wl.cpu_steps * 5))), len(Z))
    ssm = wl.oracle_ssm()
    pf = pf_oracle.SIROracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, Np=wl.n_particles, rng=np.random.default_rng(42),
                             vectorized=True)
    pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
    from threadpoolctl import threadpool_limits

    with threadpool_limits(limits=1):  # BLAS (the nx > 1 noise matmul) on one core too
        t0 = time.perf_counter()
        for t in range(steps):
            pf.step(Z[t])
        dt = time.perf_counter() - t0
    return {"value": wl.n_particles * steps / dt, "unit": "particle-steps/s", "cores": 1, "kind": "port",
            "sample": f"{wl.name} N={wl.n_particles:.0e}, 1 replicate, {steps} steps, vectorised NumPy restatement "
                      f"(oracle/pf_oracle.py vectorized=True, BLAS limited to 1 thread), {dt:.1f} s"}


def _numpy_replicate_worker(args):
    """One core's share of cpu_baseline_numpy_cores: an independent replicate (its own seed) of the
    vectorised restatement, BLAS on one thread; returns (particle-steps, seconds) of the timed steps."""
    name, rep, steps, Z, mean0, cov0, start_at = args
    from threadpoolctl import threadpool_limits

    from oracle import pf_oracle

    wl = WORKLOADS[name]()
    if name == "mat":
        wl.build(max(steps, 1), 0)  # the sensor grid the oracle's model needs
    ssm = wl.oracle_ssm()
    with threadpool_limits(limits=1):
        pf = pf_oracle.SIROracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, Np=wl.n_particles,
                                 rng=np.random.default_rng(42 + rep), vectorized=True)
        pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
        while time.time() < start_at:  # every worker starts its timed steps together
            time.sleep(0.001)
        t0 = time.perf_counter()
        for t in range(steps):
            pf.step(Z[t])
        dt = time.perf_counter() - t0
    return wl.n_particles * steps, dt


def cpu_baseline_numpy_cores(wl, Z, mean0, cov0):
    """BASELINE.md 3 for the replicate configurations: the vectorised NumPy restatement on every core
    of this process's CPU share at once, one independent replicate per core (one process each, BLAS
    on one thread), on a bounded sample; aggregate = sum of the workers' particle-steps/s."""
    import multiprocessing as mp

    cores = oracle_threads()
    steps = min(int(os.environ.get("PF_CPU_CORES_STEPS", str(max(2, wl.cpu_steps)))), len(Z))
    Zs = np.asarray(Z[:steps], float)
    start_at = time.time() + 20.0 + 0.5 * cores  # after every worker has imported and initialised
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
    with ctx.Pool(cores) as pool:
        res = pool.map(_numpy_replicate_worker, [(wl.name, r, steps, Zs, mean0, cov0, start_at) for r in range(cores)])
    rates = [n / dt for n, dt in res]
    return {"value": float(sum(rates)), "unit": "particle-steps/s", "cores": cores, "kind": "port",
            "per_core": float(np.mean(rates)), "host_cores": os.cpu_count(),
            "sample": f"{wl.name}: {cores} independent replicates of N={wl.n_particles:.0e}, one process per core "
                      f"(spawned), {steps} steps each, vectorised NumPy restatement (oracle/pf_oracle.py "
                      f"vectorized=True, BLAS 1 thread per process), timed steps started together; "
                      f"slowest worker {max(dt for _, dt in res):.1f} s"}


def oracle_threads():
    """Threads of the C/OpenMP leg: this process's CPU share.  On the GPU pool a one-GPU box is
    allotted 16 host CPUs (OMP_NUM_THREADS is set to it there); os.cpu_count() reports the whole
    node, whose other cores serve other GPUs' jobs.  Without OMP_NUM_THREADS: the affinity set."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, env or len(os.sched_getaffinity(0)))


def cpu_c1_full_run():
    """the full BASELINE config 1 run on the faithful restatement (bit-identical
    to the reference): SV log-squared wiring, N = 1000, T = 999 (simulate_sv_1d n = 1000 seed 42),
    initialize([X0], [[0.5]]), systematic at 0.5 N, PF seed 42, 1 core."""
    from oracle import pf_oracle, ssm_oracle
    from particle_filters_amd import simulators as S

    d = S.simulate_sv_1d(1000, ALPHA, SIGMA, BETA, seed=42)
    Z = np.log(d.Y[1:] ** 2)[:, None]
    ssm = ssm_oracle.sv_logsq(ALPHA, SIGMA, BETA)
    t0 = time.perf_counter()
    o = pf_oracle.build_and_run(ssm, Z, Np=1000, seed=42, mean0=[d.X[0]], cov0=[[0.5]], vectorized=False)
    dt = time.perf_counter() - t0
    rmse = float(np.sqrt(np.mean((o["means"][:, 0] - d.X[1:]) ** 2)))
    return {"value": 1000 * len(Z) / dt, "unit": "particle-steps/s", "cores": 1, "kind": "port", "seconds": dt,
            "rmse_vs_truth": rmse,
            "sample": f"BASELINE config 1 in full: SV log-squared, N=1000, T={len(Z)}, seed 42, faithful per-particle "
                      f"restatement (oracle/pf_oracle.py, bit-identical to the reference), {dt:.2f} s"}


def rmse_vs_ref(wl, Zall, truth_all, mean0, cov0, W, K, eng_means, eng_flags, precision):
    """The north-star "RMSE vs CPU ref": the fp64 oracle (the reference algorithm, oracle/) run
    on the engine's own Philox draws (replicate 0, seed 42, the same epochs: initialize, W
    warm-up steps, the K timed steps), RMSE vs truth over the timed window for both, and
    |dRMSE|.  Scalar models: the C restatement (oracle/sir_philox.c, OpenMP); others: the NumPy
    PhiloxSIROracle on a bounded number of steps."""
    from oracle import sir_philox as SP

    if wl.nx > 1:  # the NumPy oracle runs from initialize: a bounded window of the timed steps
        K = min(K, int(3e8 // (wl.n_particles * wl.nx)) - W)
        if K < 5:
            return {"skipped": f"W={W} warm-up steps x N={wl.n_particles} x nx={wl.nx} exceed the NumPy oracle budget"}
        eng_means = np.asarray(eng_means, float)[:K]
        eng_flags = np.asarray(eng_flags)[:K]
    T = W + K
    truth = np.asarray(truth_all[W:T], float).reshape(K, -1)
    bm24 = precision == "fp32"
    t0 = time.perf_counter()
    if wl.nx == 1:
        m = SP.sv_logsq_model(ALPHA, SIGMA, BETA)
        o = SP.run_scalar(m, np.asarray(Zall[:T], float).reshape(-1), N=wl.n_particles, seed=42, rep=0, ep0=2,
                          mean0=np.asarray(mean0, float).reshape(-1)[0], var0=float(np.asarray(cov0).reshape(-1)[0]),
                          bm24=bm24)
        om, of = o["means"][W:T, None], o["flags"][W:T]
        impl = f"oracle/sir_philox.c (fp64, {oracle_threads()} OpenMP threads)"
    else:
        from oracle import pf_oracle
        ssm = wl.oracle_ssm()
        o = SP.PhiloxSIROracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, seed=42, rep=0, bm24=bm24, Np=wl.n_particles,
                               vectorized=True)
        o.initialize(np.asarray(mean0, float).reshape(-1), np.asarray(cov0, float))
        r = pf_oracle.run_filter(o, np.asarray(Zall[:T], float))
        om, of = r["means"][W:T], r["flags"][W:T]
        impl = "oracle/sir_philox.py PhiloxSIROracle (NumPy, fp64)"
    dt = time.perf_counter() - t0
    em = np.asarray(eng_means, float).reshape(K, -1)
    r_e = float(np.sqrt(np.mean((em - truth) ** 2)))
    r_o = float(np.sqrt(np.mean((om - truth) ** 2)))
    # the 1e-4 tolerance is the north star's, stated for the SV model; for the large-state
    # workloads the comparison is informative: fp32-vs-fp64 rounding flips resample decisions
    # and ancestors, after which a high-dimensional filter's trajectory is Monte-Carlo noise
    return {"rmse_engine": r_e, "rmse_ref": r_o, "abs_diff": abs(r_e - r_o),
            "tolerance": 1e-4 if wl.nx == 1 else None,
            "max_abs_dmean": float(np.max(np.abs(em - om))),
            "decision_flips": int(np.sum(np.asarray(eng_flags, bool).reshape(-1) != np.asarray(of, bool))),
            "window": f"steps [{W}, {T}) after initialize (replicate 0)",
            "ref": impl + ": the reference SIR algorithm (particle_filter.py) on the engine's Philox draws",
            "ref_seconds": dt, "ref_particle_steps_per_s": wl.n_particles * T / dt,
            "ref_threads": oracle_threads() if wl.nx == 1 else 1}


def paired_free_run(name, device=0, fixture=None):
    """SURVEY 8(c)(i) for the large-state configs: the engine's native-Philox free runs of
    oracle/free_run.CONFIGS[name] (R replicates x N particles from initialize, seed 42, replicate
    ids 0..R-1, fp32) against the fp64 oracle's runs on the same draws (committed numbers,
    tests/golden/free_run_pairs.npz): per-replicate RMSE / log-likelihood / resample rate (/ OMAT),
    mean paired difference within 3 standard errors.  Returns (verdict, engine, oracle) where
    engine / oracle map each statistic to its per-replicate array."""
    from oracle import free_run as FR
    from particle_filters_amd.batch import ParticleFilterBatch

    cfg = FR.CONFIGS[name]
    T, W, nt = cfg["T"], cfg["W"], cfg.get("n_targets")
    if fixture is None:
        fixture = np.load(os.path.join(REPO, "tests", "golden", "free_run_pairs.npz"), allow_pickle=False)
    if list(fixture[f"{name}_config"]) != [cfg["R"], cfg["N"], T, W, cfg["seed"]]:
        raise ValueError(f"free_run_pairs.npz {name}: configuration differs from oracle/free_run.CONFIGS")
    wl = WORKLOADS[name]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(T, 0)
    pf = ParticleFilterBatch(g, h, Q, R, Np=cfg["N"], n_replicates=cfg["R"], seed=cfg["seed"], device=device)
    try:
        pf.initialize(mean0, cov0)
        res = pf.run(np.asarray(Z[:T], float), with_cov=False)
    finally:
        pf.close()
    truth = np.asarray(truth[:T], float)
    eng_rows, ora_rows = [], []
    for r in range(cfg["R"]):
        eng_rows.append(FR.summarise(FR.per_step(res.means[:, r], res.flags[:, r], res.log_norm[:, r], truth, nt), W))
        ora = {k: fixture[f"{name}_{k}"][r] for k in ("err2", "flags", "lse", "omat") if f"{name}_{k}" in fixture}
        ora_rows.append(FR.summarise(ora, W))
    eng = {k: np.array([s[k] for s in eng_rows]) for k in eng_rows[0]}
    ora = {k: np.array([s[k] for s in ora_rows]) for k in ora_rows[0]}
    v = FR.paired_verdict(eng, ora, name=name)
    v.update({"config": dict(cfg), "window": f"steps [{W}, {T}) after initialize",
              "oracle": "oracle/sir_philox.py PhiloxSIROracle (fp64 NumPy restatement of particle_filter.py) on the "
                        "engine's Philox draws, tests/golden/free_run_pairs.npz (make_golden_free_run.py)"})
    return v, eng, ora


def spawn_ranks(n):
    """``bench.py --gpus N`` without a launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1) before this process
    touches a GPU, wait for them, and return the worst exit code.  Rank 0 prints the line."""
    import socket
    import subprocess

    import torch

    have = torch.cuda.device_count()  # does not initialise the HIP runtime on this image
    if n > have:
        log(f"bench: --gpus {n} needs {n} HIP devices, {have} visible; refusing")
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="sv")
    ap.add_argument("--precision", choices=("fp32", "fp64"), default="fp32")
    ap.add_argument("--replicates-total", type=int, default=None,
                    help="strong scaling: this many replicates over all ranks (SURVEY 8(e): R=64 for MAT); "
                         "default: the workload's fixed replicates per GPU (weak scaling)")
    ap.add_argument("--kernel-path", choices=("auto", "runtime"), default="auto",
                    help="runtime: run the model on the runtime-shape kernels even if its shape is compiled")
    ap.add_argument("--spawn", action="store_true", help="launch the rank processes even for --gpus 1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref", action="store_true", help="skip the rmse_vs_ref oracle leg")
    ap.add_argument("--no-cov", action="store_true",
                    help="do not compute the per-step posterior covariance (the reference computes it)")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.spawn):
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # a launcher (torchrun or spawn_ranks) sets WORLD_SIZE: then the RCCL group exists even at world 1
    use_dist = "WORLD_SIZE" in os.environ
    if args.workload in ("ledh", "edh", "ledh_mat"):
        algo = "ledh" if args.workload == "ledh_mat" else args.workload
        return main_ledh(args, world, rank, local, algo=algo, use_dist=use_dist,
                         model="mat" if args.workload == "ledh_mat" else "l96")
    wl = WORKLOADS[args.workload]()
    K = args.steps if args.steps is not None else wl.defaults[0]
    W = args.warmup if args.warmup is not None else wl.defaults[1]

    import torch

    torch.cuda.set_device(local)
    dist = None
    if use_dist:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from particle_filters_amd import _native as NV
    from particle_filters_amd.batch import ParticleFilterBatch
    from particle_filters_amd.distributed import gather_summary_buffers

    # the series also covers the CPU baselines' samples (they start at the timed window)
    cpu_need = 0 if (rank != 0 or args.no_cpu_baseline) else wl.cpu_steps * 5
    # nx > 4 with the covariance: a second window of K steps times the step kernels alone
    split_cov = (not args.no_cov) and wl.nx > 4
    T_data = W + max(K * (2 if split_cov else 1), cpu_need)
    g, h, Q, R, Zall, truth_all, mean0, cov0 = wl.build(T_data, rank)
    nx, Rl, Np = wl.nx, wl.replicates, wl.n_particles
    strong = args.replicates_total is not None
    rbase = rank * Rl
    if strong:  # distributed.shard_replicates: rank r runs a contiguous block of the global replicates
        from particle_filters_amd.distributed import shard_replicates

        if args.replicates_total % world:  # the summaries' all-gather takes equal blocks per rank
            raise SystemExit(f"--replicates-total {args.replicates_total} is not a multiple of {world} ranks")
        rbase, Rl = shard_replicates(args.replicates_total, world, rank)
        wl.replicates = Rl
    dev = torch.device("cuda", local)
    rdt = torch.float32 if args.precision == "fp32" else torch.float64

    def dz(a):  # [T][nz] shared by every replicate -> [T][R][nz] in HBM, engine precision
        a = np.broadcast_to(np.asarray(a, float)[:, None, :], (a.shape[0], Rl, wl.nz))
        return torch.tensor(np.ascontiguousarray(a), dtype=rdt, device=dev).contiguous()

    # one device series for the warm-up and the timed window: the timed job's inputs, outputs and
    # gather buffers are the same allocations (the same pages) the warm-up already ran on
    dZall = dz(Zall[:W + K])
    dZw, dZ = dZall[:W], dZall[W:W + K]
    pf = ParticleFilterBatch(g, h, Q, R, Np=Np, n_replicates=Rl, replicate_base=rbase,
                             seed=42, precision=args.precision, device=local, kernel_path=args.kernel_path)
    pf.initialize(mean0, cov0)
    lib = NV.load()
    NV.check(lib.pf_set_timing(pf.handle, 1), "pf_set_timing")

    # the posterior covariance of every step (pf.py:266-267, part of the reference's reported state
    # and of the gathered summaries, distributed.SUMMARY_FIELDS); --no-cov drops it (named in config)
    ncov = 0 if args.no_cov else nx * nx
    out_store = torch.zeros(max(W, K) * Rl * (nx + ncov + 3), dtype=torch.float64, device=dev)

    def outs(T):
        """The run's outputs as views of ONE contiguous float64 buffer (means [T][R][nx], covariances
        [T][R][nx][nx], Neff, log normaliser, resample flags as int32), so that the ranks' summaries
        are gathered by a single collective with no packing kernels in the timed region.  Warm-up and
        timed outputs share the storage."""
        n = T * Rl
        o = n * (nx + ncov)
        buf = out_store[:n * (nx + ncov + 3)]
        means = buf[:n * nx].view(T, Rl, nx)
        covs = buf[n * nx:o].view(T, Rl, nx, nx) if ncov else None
        neff = buf[o:o + n].view(T, Rl)
        lnorm = buf[o + n:o + 2 * n].view(T, Rl)
        flags = buf[o + 2 * n:].view(torch.int32)[:n].view(T, Rl)
        return means, neff, flags, lnorm, buf, covs

    def unpack(flat, T):
        """[world * per-rank buffer] -> per-replicate summaries [world*R][T][nx (+ nx*nx) + 3] in
        distributed.pack_summaries' row layout (after timing)."""
        n = T * Rl
        o = n * (nx + ncov)
        rows = []
        for b in flat.view(world, -1):
            parts = [b[:n * nx].view(T, Rl, nx)]
            if ncov:
                parts.append(b[n * nx:o].view(T, Rl, ncov))
            parts.append(b[o:o + n].view(T, Rl, 1))
            parts.append(b[o + 2 * n:].view(torch.int32)[:n].view(T, Rl, 1).to(torch.float64))
            parts.append(b[o + n:o + 2 * n].view(T, Rl, 1))
            rows.append(torch.cat(parts, 2).transpose(0, 1))
        return torch.cat(rows, 0)

    def run_args(dzz, T, o):  # the ctypes arguments, built outside the timed region
        means, neff, flags, lnorm, _, cv = o
        covs = None if cv is None else NV.C.c_void_p(cv.data_ptr())
        return (pf.handle, NV.C.c_void_p(dzz.data_ptr()), None, T, 0, NV.C.c_void_p(means.data_ptr()), covs,
                NV.C.c_void_p(neff.data_ptr()), NV.C.c_void_p(flags.data_ptr()), NV.C.c_void_p(lnorm.data_ptr()))

    def run(a):
        NV.check(lib.pf_run_device(*a), "pf_run_device")

    engine_stream = torch.cuda.ExternalStream(lib.pf_stream(pf.handle), device=dev)
    done = torch.cuda.Event()

    def job(a, o, gathered):
        """One pass of the timed sequence: T filter steps (outputs written by the kernels in
        HBM, no host work) and, with a process group, ONE RCCL all-gather of every rank's
        summary buffer (distributed.gather_summary_buffers) - unpacked after the timing."""
        run(a)
        if dist is None:
            return
        done.record(engine_stream)
        torch.cuda.current_stream().wait_event(done)
        gather_summary_buffers(gathered, o[4])

    ow, ot = outs(W), outs(K)
    g_store = torch.empty(world * out_store.numel(), dtype=torch.float64, device=dev) if dist else None
    gw = g_store[:world * ow[4].numel()] if dist else None
    gt = g_store[:world * ot[4].numel()] if dist else None
    aw, at = run_args(dZw, W, ow), run_args(dZ, K, ot)
    if W > 0:  # warm-up: the same sequence ahead of the timed window (loads kernels, sets up RCCL)
        job(aw, ow, gw)
    torch.cuda.synchronize()
    NV.check(lib.pf_synchronize(pf.handle), "warm-up")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    job(at, ot, gt)
    torch.cuda.synchronize()
    # this rank's clock stops when its device is done; the closing barrier below still brackets
    # the window, and the max over ranks (all_reduce) gives the job's time without the
    # barrier's own RCCL round trip
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    NV.check(lib.pf_synchronize(pf.handle), "timed run")  # raises on a hand-off timeout / all-dead filter
    ms = NV.C.c_float()
    NV.check(lib.pf_last_run_ms(pf.handle, NV.C.byref(ms)), "pf_last_run_ms")
    device_ms = float(ms.value)  # the K-step run's filter kernels on the engine stream
    if dist:
        t = torch.tensor([elapsed, device_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())

    # posterior quality of every replicate (gathered summaries on several ranks)
    truth = np.asarray(truth_all[W:W + K], float).reshape(K, nx)
    if dist is not None:
        from particle_filters_amd.distributed import unpack_summaries

        gathered = unpack_summaries(unpack(gt, K).cpu().numpy(), nx, Np)  # every replicate's summaries
        allm = np.transpose(gathered.means, (1, 0, 2))  # [world*R][K][nx]
    else:
        allm = np.transpose(ot[0].cpu().numpy(), (1, 0, 2))
    rmse = [float(np.sqrt(np.mean((allm[r] - truth) ** 2))) for r in range(allm.shape[0])]
    omat = None
    if wl.name == "mat":  # config 4's own accuracy metric (the MAT notebook's compute_omat, p = 1)
        from particle_filters_amd.metrics import omat_series

        per_rep = [float(np.mean(omat_series(truth, allm[r], 4))) for r in range(allm.shape[0])]
        omat = {"average": float(np.mean(per_rep)), "per_replicate": per_rep, "p": 1,
                "definition": "per step: optimal assignment of the 4 estimated target positions (posterior "
                              "means' x, y) to the true ones, (1/C) sum of distances; averaged over the K "
                              "timed steps, then over replicates (reference notebook "
                              "PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb compute_omat; "
                              "its joint LEDH run reports Average OMAT 10.6974 over T = 40)",
                "from": "the RCCL-gathered posterior means" if dist is not None else "the run's posterior means"}
    local_flags = ot[2].cpu().numpy()  # [K][R] this rank's resample decisions
    means_rep0 = ot[0][:, 0].cpu().numpy()  # replicate 0's means (rmse_vs_ref)
    resample_rate = float(local_flags.mean())

    # nx > 4: the run's device time covers the step kernels AND the covariance kernels (pf_cov.h).
    # The roofline is the dominant kernel's (the step kernel): time the next K steps (the data's
    # continuation, same state) without the covariance; the difference is the covariance's cost.
    cov_ms = None
    if split_cov:
        ox = outs(K)  # the timed window's outputs were read above; the storage is reused
        ax = list(run_args(dz(Zall[W + K:W + 2 * K]), K, ox))
        ax[6] = None  # no covariance
        NV.check(lib.pf_run_device(*ax), "pf_run_device (step kernels only)")
        NV.check(lib.pf_synchronize(pf.handle), "step-kernel window")
        ms2 = NV.C.c_float()
        NV.check(lib.pf_last_run_ms(pf.handle, NV.C.byref(ms2)), "pf_last_run_ms")
        cov_ms = device_ms - float(ms2.value)
        local_flags2 = ox[2].cpu().numpy()
        device_ms_step, flags_step = float(ms2.value), local_flags2
    else:
        device_ms_step, flags_step = device_ms, None

    # live roofline of the dominant kernel: device time of the timed run
    resident = bool(lib.pf_last_run_resident(pf.handle))
    step_s = device_ms_step * 1e-3 / K
    esz = 4.0 if args.precision == "fp32" else 8.0
    base_b, res_b = 2 * esz * nx + 2 * esz, 2 * esz * nx + 12.0  # SURVEY.md 8(d) at the storage width
    alg_bytes_run = Np * (K * Rl * base_b + float((local_flags if flags_step is None else flags_step).sum()) * res_b)
    achieved = alg_bytes_run / (device_ms_step * 1e-3) / 1e9
    dyn = lib.pf_kernel_path(pf.handle) == NV.PF_PATH_RUNTIME
    # large states: group kernel; shapes outside the compiled list: the runtime-shape kernel
    streamed = bool(lib.pf_last_step_streamed(pf.handle))  # persistent many-replicate step (k_step_stream)
    kname = "k_resident" if resident else ("k_dyn_step" if dyn else ("k_step_grp" if nx >= 16 else
                                                                    ("k_step_stream" if streamed else "k_step")))
    ktmpl = wl.kernel_tmpl.split(",", 1)[1]
    if dyn:
        ktmpl = ",".join(ktmpl.split(",")[-2:])  # k_dyn_step<Real, TK, OK>
    pkey = wl.name + ("_fp64" if args.precision == "fp64" else "")  # profiles/pmc_*_<pkey>.json
    traffic, traffic_src = pmc_traffic(pkey, kname)
    G, tile, lds = pf.geometry()
    workload_desc, data_desc = wl.describe(world)
    real = "float" if args.precision == "fp32" else "double"

    if rank == 0:
        cpu = None
        errors = []
        if world == 1 and not args.no_cpu_baseline:
            s0 = truth_all[W - 1] if W > 0 else mean0  # the CPU samples start at the timed window
            try:
                cpu = cpu_baseline(wl, Zall[W:], s0, cov0)
                cpu["cores_on_host"] = os.cpu_count()
            except Exception as e:  # keep the line; the error is recorded in it
                errors.append(f"faithful port: {e!r}")
                log("cpu baseline failed:", repr(e))
            try:
                npv = cpu_baseline_numpy(wl, Zall[W:], s0, cov0)
                if cpu is None:
                    cpu = {"value": None, "unit": "particle-steps/s", "cores": 1, "kind": "port"}
                cpu["numpy_vectorised"] = npv
            except Exception as e:
                errors.append(f"numpy restatement: {e!r}")
                log("cpu numpy baseline failed:", repr(e))
            if wl.replicates > 1 and wl.nx > 1:  # the replicate configuration on every core of the box
                try:
                    if cpu is None:
                        cpu = {"value": None, "unit": "particle-steps/s", "cores": 1, "kind": "port"}
                    cpu["numpy_vectorised_all_cores"] = cpu_baseline_numpy_cores(wl, Zall[W:], s0, cov0)
                except Exception as e:
                    errors.append(f"numpy restatement on all cores: {e!r}")
                    log("cpu numpy all-cores baseline failed:", repr(e))
            if wl.name in ("sv", "sv64"):
                try:
                    c1 = cpu_c1_full_run()
                    if cpu is None:
                        cpu = {"value": None, "unit": "particle-steps/s", "cores": 1, "kind": "port"}
                    cpu["c1_full_run"] = c1
                except Exception as e:
                    errors.append(f"C1 full run: {e!r}")
                    log("C1 full run failed:", repr(e))
            if errors and cpu is not None:
                cpu["errors"] = errors
        ref = None
        if not args.no_ref:
            try:
                ref = rmse_vs_ref(wl, Zall, truth_all, mean0, cov0, W, K, means_rep0,
                                  local_flags[:, 0], args.precision)
                if wl.nx > 1 and len(rmse) > 1 and "abs_diff" in ref:
                    # large states: after the first fp32-vs-fp64 decision flip the replicate-0
                    # trajectories are independent Monte-Carlo draws, so |dRMSE| is judged
                    # against the spread of the engine's own replicates (same data, other seeds)
                    sd = float(np.std(rmse, ddof=1))
                    ref["mc_sd_rmse_over_replicates"] = sd
                    ref["abs_diff_in_mc_sd"] = ref["abs_diff"] / sd if sd > 0 else None
                if wl.nx > 1 and args.precision == "fp32" and wl.name in ("l96", "mat"):
                    # the parity verdict for the large states: paired multi-replicate free runs
                    try:
                        pv, _, _ = paired_free_run(wl.name, device=local)
                        ref["paired_free_run"] = pv
                        ref["tolerance"] = ("paired free runs: mean per-replicate difference (engine - fp64 oracle, "
                                            "same Philox draws) of every statistic within 3 standard errors and "
                                            "within the stated relative margin (oracle/free_run.MARGINS), with "
                                            "3 SE / |oracle mean| <= that margin (SURVEY 8(c)(i))")
                        ref["parity_ok"] = pv["ok"]
                    except Exception as e:
                        ref["paired_free_run"] = {"error": repr(e)}
                        log("paired free run failed:", repr(e))
                if cpu is not None and wl.nx == 1 and "ref_particle_steps_per_s" in ref:
                    th = ref["ref_threads"]
                    cpu["c_openmp"] = {"value": ref["ref_particle_steps_per_s"], "unit": "particle-steps/s",
                                       "cores": th, "host_cores": os.cpu_count(),
                                       "cores_note": "this box's CPU share (OMP_NUM_THREADS of the GPU pool); the "
                                                     "node's other cores serve its other GPUs",
                                       "extrapolated_all_host_cores": ref["ref_particle_steps_per_s"] *
                                       (os.cpu_count() or th) / th,
                                       "kind": "port",
                                       "sample": f"the rmse_vs_ref run: {Np:.0e} particles x {W + K} steps, C "
                                                 f"restatement (oracle/sir_philox.c, fp64), {ref['ref_seconds']:.1f} s"}
            except Exception as e:
                ref = {"error": repr(e)}
                log("rmse_vs_ref failed:", repr(e))
        value = Np * Rl * K * world / elapsed
        line = {
            "metric": METRIC if wl.name in ("sv", "sv64") else f"particle-steps/sec (N×T/s), {wl.name} workload",
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": data_desc,
            "config": {"workload": workload_desc, "n_particles": Np, "replicates_per_gpu": Rl,
                       "replicates_total": Rl * world,
                       "kernel_path": "runtime-shape (pf_dyn.h)" if dyn else "compiled shape",
                       "parallelism": f"replicates x{world} (independent filters per GPU"
                                      + (", RCCL all-gather of summaries)" if dist else ")"),
                       "geometry": {"tiles": G, "tile": tile, "lds_bytes": lds},
                       "posterior_cov": "none (--no-cov)" if args.no_cov else
                       ("every step, in the step kernel's records" if nx <= 4 else
                        "every step, MFMA block products over the reported rows (csrc/pf_cov.h)")},
            "rmse": rmse[0],
            "rmse_all_replicates": rmse,
            "omat": omat,
            "rmse_vs_ref": ref,
            "resample_rate": resample_rate,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         # the HBM fraction on the bytes the counters saw move (FETCH x2 + WRITE per step)
                         "traffic_gbs": None if traffic is None else traffic / step_s / 1e9,
                         "traffic_frac": None if traffic is None else traffic / step_s / 1e9 / HBM_PEAK_GBS,
                         "kernel": (f"pf::{kname}<{','.join(ktmpl.split(',')[1:])}>" if streamed
                                    else f"pf::{kname}<{real},{ktmpl}>"),
                         "steps_per_launch": K if resident else 1,
                         "algorithmic_bytes_per_step": alg_bytes_run / K,
                         "algorithmic_bytes_per_launch": alg_bytes_run / (1 if resident else K),
                         "avg_launch_us": step_s * 1e6 * (K if resident else 1), "us_per_step": step_s * 1e6,
                         "timing": "HIP events recorded by pf_run_device on the engine stream around its "
                                   "filter kernels (pf_set_timing / pf_last_run_ms)"
                                   + ("; nx > 4: the step kernels' time from a second K-step window without "
                                      "the covariance (the data's continuation), the covariance kernels' time is "
                                      "the difference" if split_cov else ""),
                         "cov_us_per_step": None if cov_ms is None else cov_ms * 1e3 / K,
                         "traffic_unit": "HBM bytes per filter step", "traffic_source": traffic_src,
                         "valu": pmc_valu(pkey, kname, step_s * 1e6)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    # orderly teardown: torch's wrapper of the engine stream and its events go
    # before the engine destroys that stream (otherwise exit-time handlers can
    # touch a destroyed stream, seen as a segfault at exit under rocprofv3)
    del done, engine_stream
    torch.cuda.synchronize()
    pf.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
