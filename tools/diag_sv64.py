"""Where the time of the many-replicate SV step (SURVEY 8(d) roofline run, 64 x 1e6) goes.

usage: python tools/diag_sv64.py [R] [N] [K]                  device ms/step at thresh 0.5 and 0 (never resample)
       PF_LIB=build/libpf_hip_stamps.so python tools/diag_sv64.py ...   + per-workgroup phase stamps of the last launch
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C

from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
Np = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lib = NV.load()
stamps = hasattr(lib, "pf_debug_stamps_sv") and "stamps" in os.environ.get("PF_LIB", "")
d = S.simulate_sv_1d(200, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)[:, None]
SL, WG = 10, 65536

for thresh in (0.5, 0.0):
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                             Np=Np, n_replicates=R, seed=42, resample_thresh=thresh)
    pf.initialize([float(d.X[0])], [[0.5]])
    NV.check(lib.pf_set_timing(pf.handle, 1), "timing")
    G, tile, lds = pf.geometry()
    pf.run(Z[:5])
    for rep in range(2):
        res = pf.run(Z[5 + rep * K:5 + (rep + 1) * K])
        ms = C.c_float()
        NV.check(lib.pf_last_run_ms(pf.handle, C.byref(ms)), "ms")
        fl = np.asarray(res.flags)
        print(f"thresh={thresh} R={R} N={Np} G={G} tile={tile} lds={lds}: {ms.value / K * 1e3:.1f} us/step "
              f"(resample decisions per step: {fl.sum() / K:.2f} of {R})", flush=True)
    if stamps:
        # stamp a fused gather launch: a run whose last step follows a resample decision and makes none
        ref = pf.run(Z[5 + 2 * K:5 + 3 * K])
        fl = np.asarray(ref.flags)
        cand = [q for q in range(1, K) if fl[q - 1].any() and not fl[q].any()]
        gath = None
        if cand and thresh > 0:
            q = cand[0]
            pf2 = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                      Np=Np, n_replicates=R, seed=42, resample_thresh=thresh)
            pf2.initialize([float(d.X[0])], [[0.5]])
            pf2.run(Z[:5 + 2 * K])
            pf2.run(Z[5 + 2 * K:5 + 2 * K + q + 1])
            gath = fl[q - 1]
            pf2.close()
        n = min(G * R, WG)
        buf = (C.c_ulonglong * (n * SL))()
        assert lib.pf_debug_stamps_sv(buf, n * SL) == 0
        full = np.array(buf[:], dtype=np.float64).reshape(n, SL)
        a = full[:, :6]
        t0 = a[:, 0].min()
        rel = (a - t0) / 100.0
        sub = (full[:, 6:9] - t0) / 100.0  # ancestors: after the prefix searches, the first tile's scan, all tiles
        ntiles = full[:, 9]
        groups = [("all", np.ones(n, bool))]
        if gath is not None:
            rg = np.repeat(np.asarray(gath, bool), G)[:n]
            groups = [(f"gathering replicates ({int(gath.sum())} of {R})", rg), ("other replicates", ~rg)]
        print(f"  last launch{' (fused gather)' if gath is not None else ''}: span {rel[:, 5].max():.1f} us")
        names = ["entry->head", "head->outputs", "->ancestors", "->chunks", "->record"]
        for gname, msk in groups:
            if not msk.any():
                continue
            life = rel[msk, 5] - rel[msk, 0]
            print(f"   {gname}: workgroup lifetime min {life.min():.2f} med {np.median(life):.2f} "
                  f"p90 {np.percentile(life, 90):.2f} max {life.max():.2f} us")
            for k, nm in enumerate(names):
                dk = rel[msk, k + 1] - rel[msk, k]
                print(f"    {nm:14s} med {np.median(dk):6.2f}  p90 {np.percentile(dk, 90):6.2f}  max {dk.max():6.2f} us")
            if gath is not None and gname.startswith("gathering"):
                pts = [rel[msk, 2], sub[msk, 0], sub[msk, 1], sub[msk, 2], rel[msk, 3]]
                for nm, (x0, x1) in zip(["  prefix search", "  1st tile scan", "  tiles rest", "  fill"],
                                        zip(pts[:-1], pts[1:])):
                    dk = x1 - x0
                    print(f"    {nm:14s} med {np.median(dk):6.2f}  p90 {np.percentile(dk, 90):6.2f}  max {dk.max():6.2f} us")
                nt = ntiles[msk]
                print(f"    source tiles per workgroup: mean {nt.mean():.2f}, max {nt.max():.0f}, "
                      f"histogram {np.bincount(nt.astype(int)).tolist()}")
        st = np.sort(rel[:, 0])
        print(f"    starts: 10% by {st[len(st) // 10]:.1f} us, 50% by {st[len(st) // 2]:.1f}, 90% by "
              f"{st[9 * len(st) // 10]:.1f}; live at t=span/2: "
              f"{int(((rel[:, 0] <= rel[:, 5].max() / 2) & (rel[:, 5] >= rel[:, 5].max() / 2)).sum())}")
    pf.close()
