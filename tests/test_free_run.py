"""CPU checks of the paired free-run parity machinery (oracle/free_run.py) and of its committed
oracle numbers (tests/golden/free_run_pairs.npz): the verdict arithmetic on synthetic pairs, the
fixture's shape against oracle/free_run.CONFIGS, and the fixture's first steps regenerated from
the oracle (so the committed numbers are the oracle's, not stale)."""

import numpy as np
import pytest

from oracle import free_run as FR
from tests.conftest import load_golden


def test_paired_verdict_arithmetic():
    rng = np.random.default_rng(0)
    o = rng.normal(1.0, 0.1, 32)
    m = {"rmse": 0.05}
    same = FR.paired_verdict({"rmse": o.copy()}, {"rmse": o}, margins=m)
    assert same["ok"] and same["rmse"]["mean_paired_diff"] == 0.0
    noisy = FR.paired_verdict({"rmse": o + rng.normal(0, 0.01, 32)}, {"rmse": o}, margins=m)
    assert noisy["ok"] and abs(noisy["rmse"]["z"]) < 3 and noisy["rmse"]["powered"]
    biased = FR.paired_verdict({"rmse": o + 0.05 + rng.normal(0, 0.01, 32)}, {"rmse": o}, margins=m)
    assert not biased["ok"] and biased["rmse"]["z"] > 3
    with pytest.raises(ValueError):
        FR.paired_verdict({"rmse": o[:3]}, {"rmse": o}, margins=m)
    with pytest.raises(ValueError):
        FR.paired_verdict({"rmse": o}, {"rmse": o})  # no margins and no configuration name


def test_paired_verdict_margin_and_power():
    """The stated margin binds even when the bias hides in the noise, and a check too noisy to see a
    bias of the margin's size fails as unpowered (oracle/free_run.py paired_verdict)."""
    rng = np.random.default_rng(1)
    o = rng.normal(1.0, 0.1, 64)
    m = {"rmse": 0.05}
    # a 6 % bias with large paired noise: within 3 SE, but over the margin and unpowered
    hidden = FR.paired_verdict({"rmse": o * 1.06 + rng.normal(0, 0.5, 64)}, {"rmse": o}, margins=m)["rmse"]
    assert not hidden["powered"] and not hidden["ok"]
    # a 6 % bias with little noise: powered, outside both the SE band and the margin
    clear = FR.paired_verdict({"rmse": o * 1.06 + rng.normal(0, 0.005, 64)}, {"rmse": o}, margins=m)["rmse"]
    assert clear["powered"] and not clear["within_margin"] and not clear["ok"]
    # a 1 % bias with little noise: powered and within the margin, but resolved by the SE band
    small = FR.paired_verdict({"rmse": o * 1.01 + rng.normal(0, 0.001, 64)}, {"rmse": o}, margins=m)["rmse"]
    assert small["powered"] and small["within_margin"] and not small["within_se"]
    assert abs(small["detectable_bias_rel"] - 3 * small["se_paired_diff"] / abs(small["oracle_mean"])) < 1e-15


def test_margins_cover_every_statistic():
    for name in FR.CONFIGS:
        need = {"rmse", "loglik", "resample_rate"} | ({"omat"} if FR.CONFIGS[name].get("n_targets") else set())
        assert need <= set(FR.MARGINS[name]), name
        assert all(0 < v <= 0.25 for v in FR.MARGINS[name].values())


def test_summarise_window_and_omat():
    T, nt = 6, 4
    truth = np.zeros((T, 16))
    means = np.ones((T, 16))
    s = FR.per_step(means, np.array([1, 0, 1, 1, 0, 0]), np.arange(T, dtype=float), truth, nt)
    assert np.allclose(s["err2"], 1.0) and np.allclose(s["omat"], np.sqrt(2.0))
    r = FR.summarise(s, 2)
    assert r["rmse"] == 1.0 and r["loglik"] == 2 + 3 + 4 + 5 and r["resample_rate"] == 0.5


def test_fixture_matches_configs():
    fx = load_golden("free_run_pairs")
    for name, cfg in FR.CONFIGS.items():
        assert list(fx[f"{name}_config"]) == [cfg["R"], cfg["N"], cfg["T"], cfg["W"], cfg["seed"]]
        assert cfg["R"] >= 16
        for k in ("err2", "flags", "lse") + (("omat",) if cfg.get("n_targets") else ()):
            assert fx[f"{name}_{k}"].shape == (cfg["R"], cfg["T"]), (name, k)
        assert np.all(np.isfinite(fx[f"{name}_lse"]))


@pytest.mark.parametrize("name,rep", [("l96", 5), ("mat", 17)])
def test_fixture_prefix_regenerates(name, rep):
    """The oracle's first 3 steps of one replicate at the full N reproduce the committed numbers
    (the later steps follow from the same code)."""
    import bench

    cfg = FR.CONFIGS[name]
    wl = bench.WORKLOADS[name]()
    _, _, _, _, Z, truth, mean0, cov0 = wl.build(cfg["T"], 0)
    s = FR.oracle_replicate(wl.oracle_ssm(), np.asarray(Z[:3], float), np.asarray(truth[:3], float), mean0, cov0,
                            N=cfg["N"], seed=cfg["seed"], rep=rep, n_targets=cfg.get("n_targets"))
    fx = load_golden("free_run_pairs")
    for k, v in s.items():
        np.testing.assert_array_equal(v, fx[f"{name}_{k}"][rep, :3], err_msg=f"{name} {k}")
