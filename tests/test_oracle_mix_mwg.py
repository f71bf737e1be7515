"""Oracle pins for GaussianRandomWalkMix / HaarioTypeAdaptation / GenericChainStats
mean-cov on the general schedule path (orc_run_mwg, kind 3): against the literal
numpy restatement (oracle/literal.py run_mwg_chain, the reference's in-place
remove/reimpose_constraints! round trips as written), and, for a single joint
update without positivity flags, against the cfg 4 restatement orc_run_mix bit
for bit (the two restatements share no code for the step)."""
import numpy as np
import pytest

from oracle import literal as LT


def compare(oracle, ups, steps, C, mu, t_sigma, obs, theta0, seed, chain_moments=False, rtol=1e-12):
    """Accept streams equal; θ, θ° within rtol (LAPACK vs the canonical order: after a
    readjust the two Cholesky factors of the same covariance differ in the last bits)."""
    D = len(mu)
    st = oracle.MWGState(np.tile(theta0, (C, 1)), mu, ups, chain_moments=chain_moments)
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=t_sigma, obs=obs, steps=steps)
    for c in range(C):
        o = LT.run_mwg_chain(seed, c, list(theta0), mu, ups, t_sigma, obs, steps, chain_moments=chain_moments)
        assert np.array_equal(np.array(o["acc"]), h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(np.array(o["theta"]), h["theta"][:, c], rtol=rtol, atol=rtol / 10)
        np.testing.assert_allclose(np.array(o["prop"]), h["prop"][:, c], rtol=rtol, atol=rtol / 10)
        np.testing.assert_allclose(o["state"], st.theta[c], rtol=rtol, atol=rtol / 10)
        for p, u in enumerate(ups):
            n = len(u["coords"])
            if u.get("haario_k"):
                hm, hc = st.haario(p, n)
                np.testing.assert_allclose(o["hmean"][p], hm[c], rtol=1e-10, atol=1e-12)
                np.testing.assert_allclose(o["hcov"][p], hc[c], rtol=1e-9, atol=1e-12)
                Lb = st.lb(p, n)[c]
                np.testing.assert_allclose(np.linalg.cholesky(o["sigma_b"][p]), Lb, rtol=1e-9, atol=1e-12)
        if chain_moments:
            np.testing.assert_allclose(o["smean"], st.smean[c], rtol=1e-10, atol=1e-12)
            np.testing.assert_allclose(o["scov"], st.scov[c], rtol=1e-9, atol=1e-12)
    assert D == st.D
    return st, h


def test_mix_with_positivity_flags_and_haario_at_d2(oracle):
    """GaussianRandomWalkMix(Σ_A, Σ_B, λ = 0.4, pos = [true, false]) + Haario(k = 25):
    the pick, the five in-place exp/log round trips of a step, register! on the
    log scale (adaptation.jl:407,412), readjusts on the log-scale covariance."""
    mu = np.array([2.0, 0.5])
    S = np.array([[0.5, 0.1], [0.1, 0.4]])
    obs = mu + np.random.default_rng(1).multivariate_normal(np.zeros(2), S, size=6)
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=0.05 * np.eye(2), sigma_b=[[0.2, 0.05], [0.05, 0.1]],
                             lam=0.4, haario_k=25, pos=[True, False])]
    st, h = compare(oracle, ups, [(i, 1) for i in range(1, 201)], 6, mu, S, obs, [1.0, 0.0], 77)
    assert np.all(h["theta"][..., 0] > 0)
    assert st.M[0] == 200 % 25


def test_mix_block_with_haario_beside_a_gaussian_block_and_chain_moments(oracle):
    """Two updates at D = 4: a mix + Haario(k = 15) block on {1, 2} registering on both
    updates' steps, a GaussianRandomWalk on {3, 4}; GenericChainStats mean/cov after
    every update step (chain_statistics.jl:46-49)."""
    rng = np.random.default_rng(2)
    mu = rng.normal(size=4)
    obs = mu + rng.normal(size=(8, 4))
    ups = [oracle.mwg_update(oracle.KIND_MIX, [0, 1], sigma=0.2 * np.eye(2), sigma_b=0.1 * np.eye(2), lam=0.5,
                             haario_k=40),
           oracle.mwg_update(2, [2, 3], sigma=0.05 * np.eye(2))]
    steps = [(i, p) for i in range(1, 201) for p in (1, 2)]
    st, _ = compare(oracle, ups, steps, 5, mu, np.eye(4), obs, list(mu), 78, chain_moments=True, rtol=1e-8)
    assert st.M[0] == 200 % 40
    assert not np.any(st.faults & 4)


def test_single_joint_mix_equals_the_cfg4_restatement(oracle):
    """P = 1, coords 1:D, no positivity flags: orc_run_mwg's kind 3 and orc_run_mix
    give the same bits (θ, accept stream, ll, L_B after readjusts, mean/cov)."""
    rng = np.random.default_rng(3)
    D, C, M = 6, 64, 150
    mu = rng.normal(size=D)
    obs = mu + rng.normal(size=(10, D))
    SA = 0.02 * np.eye(D)
    B = rng.normal(size=(D, D))
    SB = 0.02 * (B @ B.T / D + np.eye(D))
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=SA, sigma_b=SB, lam=0.5, haario_k=40)]
    st = oracle.MWGState(np.zeros((C, D)), mu, ups, chain_moments=True)
    h = oracle.run_mwg(st, ups, seed=9, t_sigma=np.eye(D), obs=obs, steps=[(i, 1) for i in range(1, M + 1)])
    ms = oracle.MixState(np.zeros((C, D)), sigma_b=SB)
    hm = oracle.run_mix(ms, seed=9, sigma_a=SA, t_sigma=np.eye(D), obs=obs, iter0=1, nsteps=M, lam=0.5, haario_k=40)
    assert np.array_equal(h["acc"], hm["acc"])
    assert np.array_equal(st.theta, ms.theta) and np.array_equal(st.ll, ms.ll)
    assert np.array_equal(st.lb(0, D), ms.LB.reshape(C, D, D))
    assert np.array_equal(st.smean, ms.mean) and np.array_equal(st.scov, ms.cov.reshape(C, D, D))
    hmn, hcv = st.haario(0, D)
    assert np.array_equal(hmn, ms.mean) and np.array_equal(hcv, ms.cov.reshape(C, D, D))
