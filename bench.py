#!/usr/bin/env python
"""Benchmark: BASELINE config 2 — SIR filter on the 1-D SV model, N = 1e6 particles.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One *step* = one filter time step (predict + weight + ESS + resample-if-needed +
posterior summary) over all N = 1,000,000 particles of one filter.  Each rank
(one process per GPU, ``torch.distributed`` over RCCL when N > 1) runs its own
independent Monte-Carlo replicate (Philox replicate id = rank) on the same
synthetic SV series; per-GPU work is fixed ("weak" scaling).  The timed region
is W-step warm-up excluded, then exactly K steps of the device-resident loop
(``pf_run_device``: inputs already in HBM, no host sync inside), followed by the
RCCL all-gather of every replicate's posterior summaries (means, ESS, flags),
bracketed by barrier + device synchronisation; the max over ranks is reported.

Extra JSON fields:
  roofline      dominant kernel: k_resident<f32, SV> — ONE launch runs all K steps
                with the particles register-resident (pf_resident.h); falls back to
                k_step (one launch per step) where the resident grid does not fit.
                achieved = algorithmic bytes per step (N x 16 B: read x, lw; write
                x, lw — SURVEY.md 8(d)) x steps per launch / the launch's device
                duration, timed live with HIP events recorded on the engine's own
                stream around the timed run; traffic = HBM bytes per step from the
                committed rocprofv3 PMC passes (profiles/pmc_traffic.json:
                FETCH_SIZE doubled per the gfx950 rule + WRITE_SIZE), or null.  The
                resident kernel keeps the state on chip, so traffic << algorithmic.
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
N_PARTICLES = 1_000_000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ALPHA, SIGMA, BETA = 0.95, 0.2, 1.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel):
    """HBM bytes per filter step of `kernel` from the committed PMC summary, if present."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        d = json.load(fh)
    if d.get("kernel_short") != kernel:
        return None, None
    return d.get("bytes_per_step"), d.get("source")


def cpu_baseline(Z, X0):
    """Faithful reference CPU path (per-particle Python g/h, particle_filter.py:237,257)
    on a bounded sample: the bench workload (N = 1e6) for a few steps, 1 core."""
    from oracle import pf_oracle, ssm_oracle

    steps = int(os.environ.get("PF_CPU_BASELINE_STEPS", "3"))
    ssm = ssm_oracle.sv_logsq(ALPHA, SIGMA, BETA)
    pf = pf_oracle.SIROracle(ssm.g, ssm.h, ssm.Q, ssm.R, Np=N_PARTICLES, rng=np.random.default_rng(42))
    pf.initialize(np.array([X0]), np.array([[0.5]]))
    t0 = time.perf_counter()
    for t in range(steps):
        pf.step(Z[t])
    dt = time.perf_counter() - t0
    return {"value": N_PARTICLES * steps / dt, "unit": "particle-steps/s", "cores": 1, "kind": "port",
            "sample": f"SV log-squared N=1e6, {steps} steps, faithful per-particle restatement "
                      f"(oracle/pf_oracle.py, bit-identical to the reference), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import particle_filters_amd as pfa
    from particle_filters_amd import _native as NV, models as M, simulators as S
    from particle_filters_amd.batch import ParticleFilterBatch

    K, W = args.steps, args.warmup
    data = S.simulate_sv_1d(W + K + 1, ALPHA, SIGMA, BETA, seed=42)
    Zall = np.log(data.Y[1:] ** 2)  # log-squared wiring (PF_VS_experiments.ipynb cell 6)
    dev = torch.device("cuda", local)
    dZw = torch.tensor(Zall[:W], dtype=torch.float32, device=dev).contiguous()
    dZ = torch.tensor(Zall[W:W + K], dtype=torch.float32, device=dev).contiguous()

    pf = ParticleFilterBatch(M.SVTransition(ALPHA), M.SVLogSqObservation(BETA), [[SIGMA ** 2]],
                             [[M.LOGCHI2_VAR]], Np=N_PARTICLES, n_replicates=1, replicate_base=rank,
                             seed=42, precision="fp32", device=local)
    pf.initialize([data.X[0]], [[0.5]])
    lib = NV.load()

    def outs(T):
        return (torch.zeros((T, 1), dtype=torch.float64, device=dev), torch.zeros((T, 1), dtype=torch.float64, device=dev),
                torch.zeros((T, 1), dtype=torch.int32, device=dev), torch.zeros((T, 1), dtype=torch.float64, device=dev))

    def run(dz, T, o):
        means, neff, flags, lnorm = o
        st = lib.pf_run_device(pf.handle, NV.C.c_void_p(dz.data_ptr()), None, T, 0,
                               NV.C.c_void_p(means.data_ptr()), None, NV.C.c_void_p(neff.data_ptr()),
                               NV.C.c_void_p(flags.data_ptr()), NV.C.c_void_p(lnorm.data_ptr()))
        NV.check(st, "pf_run_device")

    ow, ot = outs(W), outs(K)
    gathered = [torch.zeros((K, 3), dtype=torch.float64, device=dev) for _ in range(world)]

    engine_stream = torch.cuda.ExternalStream(lib.pf_stream(pf.handle), device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def job(dz, T, o):
        """One pass of the timed sequence: T filter steps + RCCL gather of the summaries."""
        ev0.record(engine_stream)
        run(dz, T, o)
        ev1.record(engine_stream)
        NV.check(lib.pf_synchronize(pf.handle))
        summary = torch.stack([o[0][:, 0], o[1][:, 0], o[2][:, 0].to(torch.float64)], dim=1)
        if summary.shape[0] < K:
            summary = torch.nn.functional.pad(summary, (0, 0, 0, K - summary.shape[0]))
        if dist:
            dist.all_gather(gathered, summary.contiguous())
        else:
            gathered[0].copy_(summary)

    # warm-up: the exact timed sequence (loads torch / RCCL kernels, clocks up the GPU)
    job(dZw if W > 0 else dZ[:1], max(W, 1), ow if W > 0 else outs(1))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    job(dZ, K, ot)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    device_ms = ev0.elapsed_time(ev1)  # device time of the K-step run on the engine stream
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # posterior quality of every replicate (gathered summaries)
    truth = data.X[W + 1:W + K + 1]
    allm = torch.stack(gathered).cpu().numpy()  # [world][K][3]
    rmse = [float(np.sqrt(np.mean((allm[r, :, 0] - truth) ** 2))) for r in range(world)]

    # live roofline of the dominant kernel: device time of the timed run
    resident = bool(lib.pf_last_run_resident(pf.handle))
    step_s = device_ms * 1e-3 / K
    alg_bytes = N_PARTICLES * 16.0  # per filter step
    achieved = alg_bytes / step_s / 1e9
    kname = "k_resident" if resident else "k_step"
    traffic, traffic_src = pmc_traffic(kname)
    G, tile, lds = pf.geometry()

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(Zall[W:], data.X[W])
                cpu["cores_on_host"] = os.cpu_count()
            except Exception as e:  # keep the bench line even if the baseline leg breaks
                log("cpu baseline failed:", repr(e))
        value = N_PARTICLES * K * world / elapsed
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (simulate_sv_1d alpha=0.95 sigma=0.2 beta=1 seed=42, log-squared wiring)",
            "config": {"workload": "SIR bootstrap PF, 1-D SV (BASELINE config 2): N=1e6 particles per GPU, "
                                   "systematic resampling at Neff<0.5N, T=steps",
                       "n_particles": N_PARTICLES, "replicates_per_gpu": 1,
                       "parallelism": f"replicates x{world} (one independent filter per GPU, RCCL all-gather of summaries)",
                       "geometry": {"tiles": G, "tile": tile, "lds_bytes": lds}},
            "rmse": rmse[0],
            "rmse_all_replicates": rmse,
            "resample_rate": float(np.mean(allm[0, :, 2])),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"pf::{kname}<float,1,1,LINEAR,LINEAR>",
                         "steps_per_launch": K if resident else 1,
                         "algorithmic_bytes_per_step": alg_bytes,
                         "algorithmic_bytes_per_launch": alg_bytes * (K if resident else 1),
                         "avg_launch_us": step_s * 1e6 * (K if resident else 1), "us_per_step": step_s * 1e6,
                         "traffic_unit": "HBM bytes per filter step", "traffic_source": traffic_src},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    # orderly teardown: torch's wrapper of the engine stream and its events go
    # before the engine destroys that stream (otherwise exit-time handlers can
    # touch a destroyed stream, seen as a segfault at exit under rocprofv3)
    del ev0, ev1, engine_stream
    torch.cuda.synchronize()
    pf.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
