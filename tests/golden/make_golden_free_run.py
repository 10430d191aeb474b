"""Generate tests/golden/free_run_pairs.npz: the oracle side of the paired multi-replicate
free-run parity check of BASELINE configs 3 (L96 d = 40) and 4 (joint 16-D acoustic tracking).

    python tests/golden/make_golden_free_run.py [--procs 8] [--only l96|mat]

For every replicate r of oracle/free_run.CONFIGS[name] the fp64 oracle (PhiloxSIROracle: the
reference algorithm of models/particle_filter.py on the engine's Philox draws, seed 42,
replicate id r, fresh-handle epochs) filters the bench workload's data (bench.py Workload.build,
the same series the GPU runs), and the per-step squared error, resample flag, log normaliser and
(config 4) OMAT are stored.  No reference code runs here: the oracle is the restatement pinned to
the reference by tests/test_oracle_golden.py.  ~75 min on 7 cores (L96 64 x 500 steps, MAT 512 x 110).
"""

from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _data(name):
    import bench
    from oracle import free_run as FR

    cfg = FR.CONFIGS[name]
    wl = bench.WORKLOADS[name]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(cfg["T"], 0)
    return wl, cfg, np.asarray(Z[:cfg["T"]], float), np.asarray(truth[:cfg["T"]], float), mean0, cov0


def _worker(args):
    name, rep = args
    from threadpoolctl import threadpool_limits

    from oracle import free_run as FR

    wl, cfg, Z, truth, mean0, cov0 = _data(name)
    t0 = time.perf_counter()
    with threadpool_limits(limits=1):
        s = FR.oracle_replicate(wl.oracle_ssm(), Z, truth, mean0, cov0, N=cfg["N"], seed=cfg["seed"], rep=rep,
                                n_targets=cfg.get("n_targets"))
    print(f"{name} replicate {rep}: {time.perf_counter() - t0:.0f} s", flush=True)
    return rep, s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--only", choices=("l96", "mat"), default=None)
    ap.add_argument("--out", default=os.path.join(HERE, "free_run_pairs.npz"))
    args = ap.parse_args()
    import multiprocessing as mp

    from oracle import free_run as FR

    names = [args.only] if args.only else list(FR.CONFIGS)
    out = {}
    if args.only and os.path.exists(args.out):
        with np.load(args.out, allow_pickle=False) as old:
            out = {k: old[k] for k in old.files if not k.startswith(args.only + "_")}
    for name in names:
        cfg = FR.CONFIGS[name]
        with mp.get_context("spawn").Pool(args.procs) as pool:
            res = dict(pool.map(_worker, [(name, r) for r in range(cfg["R"])]))
        for k in res[0]:
            out[f"{name}_{k}"] = np.stack([res[r][k] for r in range(cfg["R"])])
        out[f"{name}_config"] = np.array([cfg["R"], cfg["N"], cfg["T"], cfg["W"], cfg["seed"]], np.int64)
    np.savez_compressed(args.out, **out)
    print("wrote", args.out, sorted(out))


if __name__ == "__main__":
    main()
