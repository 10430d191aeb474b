"""Wall-time anatomy of the bench's K=20 job (SV, N=1e6): host-side cost around one
pf_run_device launch.  Prints per-variant wall us per 20-step run (median of many runs)
next to the device time of the same runs (pf_last_run_ms).

    python tools/diag_wall.py          (PF_NO_ORDER=1: without the grid-order event)
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    from particle_filters_amd import _native as NV, models as M, simulators as S
    from particle_filters_amd.batch import ParticleFilterBatch

    torch.cuda.set_device(0)
    K, reps = 20, 60
    data = S.simulate_sv_1d(K * (reps + 4) + 2, 0.95, 0.2, 1.0, seed=42)
    Z = np.log(data.Y[1:] ** 2)[:, None]
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                             Np=1_000_000, seed=42)
    pf.initialize([data.X[0]], [[0.5]])
    lib = NV.load()
    dev = torch.device("cuda", 0)
    dZ = torch.tensor(Z[:, None, :], dtype=torch.float32, device=dev)
    n = K
    buf = torch.zeros(n * 4, dtype=torch.float64, device=dev)
    means, neff, lnorm = buf[:n], buf[n:2 * n], buf[2 * n:3 * n]
    flags = buf[3 * n:].view(torch.int32)[:n]
    args = [NV.C.c_void_p(t.data_ptr()) for t in (means, neff, flags, lnorm)]
    off = [0]

    def run():
        z = dZ[off[0]:off[0] + K]
        off[0] = (off[0] + K) % (K * reps)
        NV.check(lib.pf_run_device(pf.handle, NV.C.c_void_p(z.data_ptr()), None, K, 0, args[0], None, args[1],
                                   args[2], args[3]), "run")

    def measure(label, timing, sync):
        NV.check(lib.pf_set_timing(pf.handle, 1 if timing else 0), "timing")
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        walls, devs, launch = [], [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run()
            t1 = time.perf_counter()
            sync()
            t2 = time.perf_counter()
            walls.append((t2 - t0) * 1e6)
            launch.append((t1 - t0) * 1e6)
            if timing:
                ms = NV.C.c_float()
                NV.check(lib.pf_last_run_ms(pf.handle, NV.C.byref(ms)), "ms")
                devs.append(ms.value * 1e3)
        NV.check(lib.pf_synchronize(pf.handle), "sync")
        print(f"{label:34s} wall {np.median(walls):7.1f} us  host call {np.median(launch):6.1f} us  "
              f"device {np.median(devs) if devs else float('nan'):7.1f} us", flush=True)

    tag = " [PF_NO_ORDER=1]" if os.environ.get("PF_NO_ORDER") == "1" else ""
    modes = {"0": "markers", "1": "dispatch events", "2": "dispatch start, marker stop", "3": "marker start, dispatch stop"}
    for rnd in range(2):
        for m, name in modes.items():
            os.environ["PF_EXT_EVENTS"] = m
            measure(f"timing on ({name}){tag}", True, torch.cuda.synchronize)
        measure(f"timing off, torch sync{tag}", False, torch.cuda.synchronize)
    os.environ["PF_EXT_EVENTS"] = "1"
    measure(f"timing off, pf_synchronize{tag}", False, lambda: lib.pf_synchronize(pf.handle))
    pf.close()


if __name__ == "__main__":
    main()
