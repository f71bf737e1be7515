"""The oracle reproduces the committed golden fixtures bit for bit
(tests/golden/make_golden.py documents how they were made)."""
import numpy as np
import pytest


@pytest.mark.parametrize("name", ["gsn_d2_reftest", "gsn_d2_iso", "gsn_d32_perobs", "gsn_d32_suffstat"])
def test_oracle_reproduces_fixture(oracle, golden_dir, name):
    g = np.load(golden_dir / f"{name}.npz", allow_pickle=False)
    C, D = g["theta"].shape
    st = oracle.OracleState(np.broadcast_to(g["theta_init"], (C, D)).copy())
    h = oracle.run_gsn(st, seed=int(g["seed"]), rw_sigma=g["rw_sigma"], t_sigma=g["t_sigma"], obs=g["obs"],
                       iter0=1, nsteps=g["acc_hist"].shape[0], ll_mode=int(g["ll_mode"]))
    assert np.array_equal(h["acc"], g["acc_hist"])
    assert np.array_equal(h["ll"], g["ll_hist"])
    assert np.array_equal(h["theta"], g["theta_hist"])
    assert np.array_equal(h["prop"], g["prop_hist"])
    assert np.array_equal(st.ra, g["ra"])
    assert np.array_equal(st.nacc, g["nacc"])


def test_resume_equals_one_shot(oracle, golden_dir):
    """run! split at an arbitrary iteration continues the same stream (counter-based RNG)."""
    g = np.load(golden_dir / "gsn_d32_perobs.npz", allow_pickle=False)
    C, D = g["theta"].shape
    st = oracle.OracleState(np.zeros((C, D)))
    kw = dict(seed=int(g["seed"]), rw_sigma=g["rw_sigma"], t_sigma=g["t_sigma"], obs=g["obs"], ll_mode=0)
    h1 = oracle.run_gsn(st, iter0=1, nsteps=77, **kw)
    h2 = oracle.run_gsn(st, iter0=78, nsteps=123, **kw)
    assert np.array_equal(np.concatenate([h1["acc"], h2["acc"]]), g["acc_hist"])
    assert np.array_equal(st.theta, g["theta"])
    assert np.array_equal(st.ra, g["ra"])


def test_sharding_equals_unsharded(oracle, golden_dir):
    """Chains keyed by global id: a shard starting at chain0 = 5 reproduces chains 5..7."""
    g = np.load(golden_dir / "gsn_d32_perobs.npz", allow_pickle=False)
    st = oracle.OracleState(np.zeros((3, 32)))
    h = oracle.run_gsn(st, seed=int(g["seed"]), rw_sigma=g["rw_sigma"], t_sigma=g["t_sigma"], obs=g["obs"],
                       iter0=1, nsteps=200, chain0=5)
    assert np.array_equal(h["acc"], g["acc_hist"][:, 5:8])
    assert np.array_equal(st.theta, g["theta"][5:8])


def test_mwg_reference_workload_fixture(oracle, golden_dir):
    """The general-schedule oracle reproduces the committed reference-test fixture."""
    g = np.load(golden_dir / "mwg_d2_reftest.npz")
    steps = [tuple(int(v) for v in s) for s in g["steps"]]
    for tag, eps, ad in (("plain", 1.0, None),
                         ("adapt", 0.1, {"k": 50, "target": 0.234, "scale": 0.1, "min": 1e-12, "max": 1e7,
                                          "offset": 1e2})):
        ups = [oracle.mwg_update(1, [0], eps=[eps], adapt=ad), oracle.mwg_update(1, [1], eps=[eps], adapt=ad)]
        st = oracle.MWGState(np.zeros((8, 2)), g["mu0"], ups)
        h = oracle.run_mwg(st, ups, seed=int(g["seed"]), t_sigma=g["t_sigma"], obs=g["obs"], steps=steps)
        assert np.array_equal(h["acc"], g[f"{tag}_acc"])
        assert np.array_equal(h["theta"], g[f"{tag}_theta"])
        assert np.array_equal(h["ll"], g[f"{tag}_ll"])
        assert np.array_equal(st.ra, g[f"{tag}_ra"])
        assert np.array_equal(st.eps[:, :, 0], g[f"{tag}_eps"])
