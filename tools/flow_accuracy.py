"""Accuracy of the per-particle LEDH flow algebra on the MAT golden case (tests/golden/ledh_runs.npz,
mat_joint: the reference's joint 16-D / 25-sensor LEDH run), against a 40-digit recomputation.

    python tools/flow_accuracy.py [particle ...]   (default: 0, the most ill-conditioned, and 1, 2)

For a particle's first filter step (its x0, the reference's recorded process noise, the tracker
covariance P_0, L = n_lambda pseudo-time steps of ledh.py:136-171) the flow is integrated three ways:
  exact  mpmath at 40 digits, the reference's formulas (S solve, A = -1/2 P H^T S^{-1} H, b, eta);
  ref    the reference's fp64 formulas (numpy.linalg.solve on S);
  qr     the engine's k_flow_wave_lr algebra (pf_ledh_kernels.h): Rq = the Cholesky factor of the Gram
         W = U^T U of U = R^{-1/2} H8, the 8 x 8 system D X = Rq, K = -1/2 Rq^T X and the update carried
         in the position space
         (eta += dlam P_{:,pos} (om + 2 lam K P_pp om + K eta_pos), om = r8 + K (lam P_pp r8 + eta0_pos));
  hh     the same with Rq from a Householder QR of U (the kernel's fallback when W is not numerically
         positive definite; its primary path before the Gram / Cholesky form);
  wood   the Woodbury form through W = H8^T R^{-1} H8 (tried first, not kept).
Prints each fp64 path's max relative error of the final eta against the exact one.  This is the
evidence for the acoustic LEDH parity tolerances in tests/test_gpu_ledh.py.
"""
import os
import sys

import mpmath as mp
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = np.load(os.path.join(REPO, "tests", "golden", "ledh_runs.npz"))
M = np.load(os.path.join(REPO, "tests", "golden", "mat_data.npz"))
pj, dj = float(M["meta"][2]), float(M["meta"][3])
S = M["S"]
NX, NZ, NR = 16, 25, 8
POS = [4 * (a // 2) + (a % 2) for a in range(NR)]
F = np.array([[1, 0, 1, 0], [0, 1, 0, 1], [0, 0, 1, 0], [0, 0, 0, 1.0]])
z = g["mat_joint__Z"][0]
P = g["mat_joint__tracker_P"][0]
P = 0.5 * (P + P.T)
L = int(g["mat_joint__n_lambda"])
RD = 0.01 * np.ones(NZ)  # R = 0.1^2 I (the notebook's wiring)


def gfun(x):
    return np.concatenate([F @ x[4 * c:4 * c + 4] for c in range(4)])


def jac(eta, mpm=False):
    H = mp.zeros(NZ, NX) if mpm else np.zeros((NZ, NX))
    hv = mp.zeros(NZ, 1) if mpm else np.zeros(NZ)
    for c in range(4):
        for s in range(NZ):
            dx, dy = eta[4 * c] - S[s, 0], eta[4 * c + 1] - S[s, 1]
            den = dx * dx + dy * dy + dj
            hv[s] += pj / den
            H[s, 4 * c] = -2 * pj * dx / den ** 2
            H[s, 4 * c + 1] = -2 * pj * dy / den ** 2
    return H, hv


def householder_r(U):
    """The kernel's Householder QR (k_flow_wave_lr): per reflector all reductions at once,
    v^T v = 2 alpha (alpha - x_p), v^T u_c = x^T u_c - alpha u_{p,c}."""
    U = U.copy()
    m = U.shape[1]
    for p in range(m):
        x = U[p:, p].copy()
        nrm2, xp = np.sum(x * x), x[0]
        dots = {c: np.sum(x * U[p:, c]) for c in range(p + 1, m)}
        alpha = -np.sqrt(nrm2) if xp >= 0 else np.sqrt(nrm2)
        v = x.copy()
        v[0] = xp - alpha
        vtv = 2.0 * alpha * (alpha - xp)
        if vtv > 0:
            for c in range(p + 1, m):
                sc = dots[c] - alpha * U[p, c]
                U[p:, c] -= (2.0 / vtv) * v * sc
        U[p, p], U[p + 1:, p] = alpha, 0.0
    return U[:m]


def flow(eta0, mode):
    I = np.eye(NX)
    eta, lam, dl = eta0.copy(), 0.0, 1.0 / L
    for _ in range(L):
        lam = min(1.0, lam + dl)
        H, hv = jac(eta)
        e = hv - H @ eta
        if mode == "ref":
            A = -0.5 * P @ H.T @ np.linalg.solve(lam * H @ P @ H.T + np.diag(RD), H)
        else:
            H8, Ppp = H[:, POS], P[np.ix_(POS, POS)]
            A = np.zeros((NX, NX))
            if mode in ("qr", "hh"):  # the kernel's update in the position space (A = P_{:,pos} K E)
                U = H8 / np.sqrt(RD)[:, None]
                Rq = np.linalg.cholesky(U.T @ U).T if mode == "qr" else householder_r(U)
                X = np.linalg.solve(np.eye(NR) + lam * Rq @ Ppp @ Rq.T, Rq)
                K = -0.5 * (Rq.T @ X)
                r8 = H8.T @ ((z - e) / RD)
                om = r8 + K @ (lam * Ppp @ r8 + eta0[POS])
                eta = eta + dl * (P[:, POS] @ ((om + 2 * lam * K @ (Ppp @ om)) + K @ eta[POS]))
                continue
            else:
                W = H8.T @ (H8 / RD[:, None])
                A[:, POS] = -0.5 * P[:, POS] @ (W @ np.linalg.inv(np.eye(NR) + lam * Ppp @ W))
        c = P @ H.T @ ((z - e) / RD)
        b = (I + 2 * lam * A) @ ((I + lam * A) @ c + A @ eta0)
        eta = eta + dl * (A @ eta + b)
    return eta


def flow_exact(eta0):
    mp.mp.dps = 40
    Pm, e0 = mp.matrix(P.tolist()), mp.matrix(eta0.tolist())
    eta, lam, dl = e0.copy(), mp.mpf(0), mp.mpf(1) / L
    Rm, I, zz = mp.diag([mp.mpf("0.01")] * NZ), mp.eye(NX), mp.matrix(z.tolist())
    for _ in range(L):
        lam = min(mp.mpf(1), lam + dl)
        H, hv = jac(eta, True)
        e = hv - H * eta
        A = -mp.mpf("0.5") * Pm * H.T * (mp.inverse(lam * H * Pm * H.T + Rm) * H)
        c = Pm * H.T * (mp.inverse(Rm) * (zz - e))
        b = (I + 2 * lam * A) * ((I + lam * A) * c + A * e0)
        eta = eta + dl * (A * eta + b)
    return np.array([float(t) for t in eta])


if __name__ == "__main__":
    parts = [int(a) for a in sys.argv[1:]] or [0, 1, 2]
    for i in parts:
        eta0 = gfun(g["mat_joint__init_particles"][i]) + g["mat_joint__rng_noise"][0][i]
        H, _ = jac(eta0)
        cond = np.linalg.cond((1.0 / L) * H @ P @ H.T + np.diag(RD))
        ex = flow_exact(eta0)
        errs = {m: float(np.abs(flow(eta0, m) - ex).max() / np.abs(ex).max()) for m in ("ref", "qr", "hh", "wood")}
        print(f"particle {i}: cond(S_1) {cond:.3e}; max rel error of the final eta vs 40 digits: "
              + ", ".join(f"{m} {v:.2e}" for m, v in errs.items()), flush=True)
