"""Diagnostic: register-resident whole-run kernel (k_resident) vs the
launch-per-step path (k_step, PF_RESIDENT=0) on identical Philox noise.

Prints, per N: resample-flag agreement, first disagreement, max |dmean| /
rel dNeff / |dlse| before it, RMSE vs truth of both, and device time per step.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

lib = NV.load()


def run(N, Z, X0, resident, T, reg=False, R=1):
    os.environ["PF_RESIDENT"] = "1" if resident else "0"
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N,
                             n_replicates=R, seed=42, regularize_after_resample=reg)
    pf.initialize([X0], [[0.5]])
    dev = torch.device("cuda", 0)
    dZ = torch.tensor(np.repeat(Z[:T, None], R, axis=1), dtype=torch.float32, device=dev).contiguous()
    o = [torch.zeros((T, R), dtype=torch.float64, device=dev) for _ in range(2)]
    fl = torch.zeros((T, R), dtype=torch.int32, device=dev)
    ln = torch.zeros((T, R), dtype=torch.float64, device=dev)
    cov = torch.zeros((T, R), dtype=torch.float64, device=dev)
    st = torch.cuda.ExternalStream(lib.pf_stream(pf.handle), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    NV.check(lib.pf_run_device(pf.handle, NV.C.c_void_p(dZ.data_ptr()), None, T, 0, NV.C.c_void_p(o[0].data_ptr()),
                               NV.C.c_void_p(cov.data_ptr()), NV.C.c_void_p(o[1].data_ptr()),
                               NV.C.c_void_p(fl.data_ptr()), NV.C.c_void_p(ln.data_ptr())), "run")
    e1.record(st)
    NV.check(lib.pf_synchronize(pf.handle), "sync")
    ms = e0.elapsed_time(e1)
    parts = pf.particles()[0, :, 0]
    w = pf.weights()[0]
    return dict(mean=o[0].cpu().numpy(), neff=o[1].cpu().numpy(), flag=fl.cpu().numpy(), lse=ln.cpu().numpy(),
                cov=cov.cpu().numpy(), ms=ms, post_mean=float(np.sum(w * parts)))


def compare(N, T, reg=False, R=1):
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
    Z = np.log(d.Y[1:] ** 2)
    a = run(N, Z, d.X[0], True, T, reg, R)
    b = run(N, Z, d.X[0], False, T, reg, R)
    fa, fb = a["flag"][:, 0], b["flag"][:, 0]
    dis = np.nonzero(fa != fb)[0]
    k = dis[0] if dis.size else T
    dm = np.max(np.abs(a["mean"][:k, 0] - b["mean"][:k, 0])) if k else 0.0
    dn = np.max(np.abs(a["neff"][:k, 0] / b["neff"][:k, 0] - 1)) if k else 0.0
    dl = np.max(np.abs(a["lse"][:k, 0] - b["lse"][:k, 0])) if k else 0.0
    dc = np.max(np.abs(a["cov"][:k, 0] - b["cov"][:k, 0])) if k else 0.0
    ra = np.sqrt(np.mean((a["mean"][:, 0] - d.X[1:T + 1]) ** 2))
    rb = np.sqrt(np.mean((b["mean"][:, 0] - d.X[1:T + 1]) ** 2))
    print(f"N={N} T={T} reg={reg} R={R}: flags {int(fa.sum())}/{int(fb.sum())} agree={np.mean(fa == fb):.4f} "
          f"first_dis={k} | before: max|dmean|={dm:.2e} max|dcov|={dc:.2e} rel dNeff={dn:.2e} |dlse|={dl:.2e} | "
          f"rmse {ra:.6f} vs {rb:.6f} | post-run mean {a['post_mean']:.6f} vs {b['post_mean']:.6f} | "
          f"us/step resident {1e3 * a['ms'] / T:.2f} kstep {1e3 * b['ms'] / T:.2f}", flush=True)


def time_only(N, T, reps=3):
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
    Z = np.log(d.Y[1:] ** 2)
    for _ in range(reps):
        a = run(N, Z, d.X[0], True, T)
        rm = np.sqrt(np.mean((a["mean"][:, 0] - d.X[1:T + 1]) ** 2))
        print(f"{os.environ.get('PF_LIB', 'default lib')}: N={N} T={T} resident {1e3 * a['ms'] / T:.2f} us/step "
              f"rmse {rm:.6f} resamples {int(a['flag'].sum())}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "time":
        time_only(int(sys.argv[2]), int(sys.argv[3]))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "parts":
        particles_after_first_resample(int(sys.argv[2]))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "steps":
        steps(int(sys.argv[2]), int(sys.argv[3]))
        return
    compare(4096 * 3 + 5, 300)
    compare(1000, 300, reg=True)
    compare(10007, 300, reg=True, R=3)
    compare(1_000_000, 1000)
    compare(1_000_000, 1000)


def steps(N, T):
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
    Z = np.log(d.Y[1:] ** 2)
    a = run(N, Z, d.X[0], True, T)
    b = run(N, Z, d.X[0], False, T)
    for t in range(T):
        print(f"  t={t} mean {a['mean'][t, 0]:.8f} {b['mean'][t, 0]:.8f} neff {a['neff'][t, 0]:.3f} "
              f"{b['neff'][t, 0]:.3f} lse {a['lse'][t, 0]:.6f} {b['lse'][t, 0]:.6f} flag {a['flag'][t, 0]} "
              f"{b['flag'][t, 0]}", flush=True)


def particles_after_first_resample(N):
    T = 300
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
    Z = np.log(d.Y[1:] ** 2)
    b = run(N, Z, d.X[0], False, T)
    f = int(np.nonzero(b["flag"][:, 0])[0][0])
    out = {}
    for res in (True, False):
        os.environ["PF_RESIDENT"] = "1" if res else "0"
        pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                 Np=N, seed=42)
        pf.initialize([d.X[0]], [[0.5]])
        r = pf.run(Z[:f + 1, None])
        out[res] = (pf.particles()[0, :, 0], pf.weights()[0], r)
    xa, xb = out[True][0], out[False][0]
    bad = np.nonzero(xa != xb)[0]
    print(f"N={N}: first resample at step {f}; particles differing after it: {bad.size}/{N}; "
          f"max|dx|={np.max(np.abs(xa - xb)):.3e}; flags {out[True][2].flags[:, 0].sum()} {out[False][2].flags[:, 0].sum()}")
    print("  first bad idx", bad[:10], "values res", xa[bad[:5]], "kstep", xb[bad[:5]])
    print("  sorted equal:", np.array_equal(np.sort(xa), np.sort(xb)), "unique res/kstep", np.unique(xa).size,
          np.unique(xb).size)
    print("  means at f:", out[True][2].means[f, 0, 0], out[False][2].means[f, 0, 0],
          "neff", out[True][2].neff[f, 0], out[False][2].neff[f, 0])


if __name__ == "__main__":
    main()
