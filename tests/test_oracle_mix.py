"""Oracle pins for row f1 (BASELINE cfg 4): GaussianRandomWalkMix,
HaarioTypeAdaptation and the GenericChainStats running mean/cov.  The C
restatement orc_run_mix against the literal numpy restatement
(oracle/literal.py run_mix_chain: LAPACK Cholesky at every call, numpy outer
products), against orc_run_gsn (mix off), and against the closed-form sample
moments."""
import numpy as np
import pytest

from extensible_mcmc import workloads as W
from oracle import literal as LT


def _w(D, C=8):
    w = W.cfg2(C, D=D)
    return w, np.asarray(w.rw_sigma)


@pytest.mark.parametrize("D,lam,k", [(2, 0.5, 0), (4, 0.3, 25), (8, 0.5, 50), (8, 1.0, 40)])
def test_mix_matches_literal(oracle, D, lam, k):
    """random_walk.jl:193-232 + adaptation.jl:372-426 + chain_statistics.jl:41-66."""
    w, sa = _w(D)
    sb = 0.25 * sa
    C, S = 6, 400
    st = oracle.MixState(np.zeros((C, D)), sigma_b=sb)
    h = oracle.run_mix(st, seed=w.seed, sigma_a=sa, t_sigma=w.t_sigma, obs=np.asarray(w.obs)[:, :D], iter0=1,
                       nsteps=S, lam=lam, haario_k=k)
    for c in range(C):
        o = LT.run_mix_chain(w.seed, c, np.zeros(D), sa, sb, lam, w.t_sigma[:D, :D], np.asarray(w.obs)[:, :D], S,
                             haario_k=k)
        assert np.array_equal(o["acc"], h["acc"][:, c]), f"chain {c}: accept stream"
        np.testing.assert_allclose(o["theta"], h["theta"][:, c], rtol=1e-11, atol=1e-12)
        fin = np.isfinite(o["ll"])
        np.testing.assert_allclose(o["ll"][fin], h["ll"][fin, c], rtol=1e-12)
        np.testing.assert_allclose(o["cov"], st.cov[c], rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(o["mean"], st.mean[c], rtol=1e-11, atol=1e-14)
        np.testing.assert_allclose(o["ra"][-1], st.ra[c], rtol=1e-13)
        if k:
            np.testing.assert_allclose(np.linalg.cholesky(o["sigma_b"]), st.LB[c], rtol=1e-10, atol=1e-14)
    assert st.N == S + 1 and st.M == (S % k if k else 0)


def test_mix_off_equals_single_gaussian_update(oracle):
    """mix = 0 is GaussianRandomWalk(Σ_A) plus moments: same bits as orc_run_gsn."""
    w, sa = _w(16, 32)
    st = oracle.MixState(np.zeros((32, 16)))
    h = oracle.run_mix(st, seed=w.seed, sigma_a=sa, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=150, mix=False)
    so = oracle.OracleState(np.zeros((32, 16)))
    ho = oracle.run_gsn(so, seed=w.seed, rw_sigma=sa, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=150)
    for key in ("acc", "theta", "prop", "ll"):
        assert np.array_equal(h[key], ho[key])
    assert np.array_equal(st.ra, so.ra) and np.array_equal(st.nacc, so.nacc)


def test_chain_moments_are_sample_moments(oracle):
    """chain_statistics.jl:46-49: the recurrence is the running mean and the
    (N−1)-normalised covariance of {0 (phantom), θ_1, …, θ_S}."""
    w, sa = _w(8, 16)
    S = 300
    st = oracle.MixState(np.zeros((16, 8)), sigma_b=sa)
    h = oracle.run_mix(st, seed=w.seed, sigma_a=sa, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S)
    xs = np.concatenate([np.zeros((1, 16, 8)), h["theta"]], axis=0)
    m = xs.mean(axis=0)
    v = np.einsum("sci,scj->cij", xs - m, xs - m) / S
    np.testing.assert_allclose(st.mean, m, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(st.cov, v, rtol=1e-9, atol=1e-14)
    assert np.array_equal(st.cov, np.transpose(st.cov, (0, 2, 1)))  # exactly symmetric


def test_split_runs_equal_one_run(oracle):
    """Carried state (N, M, L_B, moments) across calls gives the same bits."""
    w, sa = _w(4, 12)
    kw = dict(seed=w.seed, sigma_a=sa, t_sigma=w.t_sigma, obs=np.asarray(w.obs)[:, :4], lam=0.4, haario_k=30)
    a = oracle.MixState(np.zeros((12, 4)), sigma_b=sa)
    ha = oracle.run_mix(a, iter0=1, nsteps=170, **kw)
    b = oracle.MixState(np.zeros((12, 4)), sigma_b=sa)
    parts = [oracle.run_mix(b, iter0=i0, nsteps=n, **kw) for i0, n in ((1, 29), (30, 1), (31, 70), (101, 70))]
    assert np.array_equal(np.concatenate([p["acc"] for p in parts]), ha["acc"])
    for key in ("theta", "ll", "ra", "mean", "cov", "LB"):
        assert np.array_equal(getattr(a, key), getattr(b, key)), key
    assert (a.N, a.M) == (b.N, b.M)


def test_posdef_failure_keeps_previous_factor(oracle):
    """readjust after 3 steps at D = 8: cov has rank ≤ 4, its Cholesky fails for
    (almost) every chain → fault bit 4 and L_B unchanged (the reference throws
    PosDefException at the next MvNormal(θ, Σ_B))."""
    w, sa = _w(8, 64)
    st = oracle.MixState(np.zeros((64, 8)), sigma_b=sa)
    L0 = st.LB.copy()
    oracle.run_mix(st, seed=w.seed, sigma_a=sa, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=3, haario_k=3)
    bad = (st.faults & 4) != 0
    assert bad.sum() >= 32
    assert np.array_equal(st.LB[bad], L0[bad])
    assert not np.array_equal(st.LB[~bad], L0[~bad]) or (~bad).sum() == 0


def test_mixture_density_extremes(oracle):
    """exp/log over the whole range (orc_exp_any / orc_log_any, the device's
    exp_any / log_any): subnormal, overflow and zero cases."""
    x = np.array([-800.0, -745.0, -740.0, -708.5, -700.0, -1.0, 0.0, 1.0, 700.0, 709.7, 710.0])
    got = oracle.exp_any_vec(x)
    with np.errstate(over="ignore"):
        ref = np.exp(x)
    fin = ref > 0
    np.testing.assert_allclose(got[fin & (ref > 1e-300) & np.isfinite(ref)], ref[fin & (ref > 1e-300) & np.isfinite(ref)],
                               rtol=2e-16)
    assert got[0] == 0.0 and np.isinf(got[-1])
    assert 0.0 < got[1] < 1e-320  # subnormal
    y = oracle.log_any_vec(np.array([0.0, 5e-324, 1e-310, 1.0, np.inf]))
    assert y[0] == -np.inf and y[-1] == np.inf and y[3] == 0.0
    np.testing.assert_allclose(y[1:3], np.log([5e-324, 1e-310]), rtol=1e-15)
