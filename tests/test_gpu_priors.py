"""Priors on the device (priors.jl:18-88) and the proposal! resample loop
(updates.jl:191-196), bit for bit against the oracle (orc_run_mwg): the
reference's test problem with ProductPrior / StandardPrior / ImproperPosPrior,
forced resampling, and D = 32 schedules on the wide general kernel (two blocks
of 16, a joint correlated Σ), including sub_ws°.ll (the ll° of REPLCallback)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W

from test_gpu_mwg import check, full_steps, run_both

pytestmark = pytest.mark.gpu

N_, U_, E_, G_ = L.DIST_NORMAL, L.DIST_UNIFORM, L.DIST_EXPONENTIAL, L.DIST_GAMMA


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


@pytest.mark.parametrize("prior", ["product", "standard", "improper_pos"])
def test_reference_problem_with_priors(oracle, prior):
    """test/runtests.jl:87-114 (D = 2, two single-site updates) with priors on each update."""
    w = W.ref_test()
    if prior == "product":
        pk, fs = [L.PRIOR_PRODUCT, L.PRIOR_PRODUCT], [[(N_, 1, 1.0, 0.5)], [(G_, 1, 4.0, 0.5)]]
    elif prior == "standard":
        pk, fs = [L.PRIOR_STANDARD, L.PRIOR_STANDARD], [[(U_, 1, -3.0, 3.0)], [(E_, 1, 2.0, 0.0)]]
    else:
        pk, fs = [L.PRIOR_IMPROPER_POS, L.PRIOR_IMPROPER_POS], [None, None]
    ups = [oracle.mwg_update(1, [0], eps=[0.8], prior=pk[0], factors=fs[0], pos=[prior == "improper_pos"]),
           oracle.mwg_update(2, [1], sigma=[[0.6]], prior=pk[1], factors=fs[1], pos=[prior == "improper_pos"])]
    steps = full_steps(300, 2)
    th0 = np.full((1000, 2), 0.5)
    eng, st, h = run_both(oracle, 2, 1000, 300, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed, theta0=th0)
    check(oracle, eng, st, h, steps, ups, 2)
    assert 0.05 < h["acc"].mean() < 0.95


def test_resampling_outside_the_support(oracle):
    """A Uniform(−0.3, 0.3) × Uniform(1.7, 2.3) prior with proposals ~10× wider than the
    support: most draws are resampled (counter blocks (r << 16) | j/2), every accepted
    state stays inside, and the streams match the oracle bitwise."""
    w = W.ref_test()
    fs = [(U_, 1, -0.3, 0.3), (U_, 1, 1.7, 2.3)]
    ups = [oracle.mwg_update(2, [0, 1], sigma=[[4.0, 0.0], [0.0, 4.0]], prior=L.PRIOR_PRODUCT, factors=fs)]
    steps = full_steps(200, 1)
    th0 = np.tile([0.0, 2.0], (512, 1))
    eng, st, h = run_both(oracle, 2, 512, 200, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed, theta0=th0)
    check(oracle, eng, st, h, steps, ups, 1)
    assert np.all(np.abs(h["prop"][..., 0]) <= 0.3) and np.all(np.abs(h["prop"][..., 1] - 2.0) <= 0.3)
    assert not np.any(st.faults & L.FAULT_PRIOR_RESAMPLES)


@pytest.mark.parametrize("ll_mode", [0, 1])
def test_d32_two_blocks_with_priors_on_the_wide_kernel(oracle, ll_mode):
    """Metropolis-within-Gibbs at the headline D = 32: two GaussianRandomWalk blocks of
    16 coordinates, a ProductPrior of Normal/Gamma factors on one and a StandardPrior of
    Exponentials on the other (so a Gaussian target at μ* > 0 keeps mass in the support)."""
    w = W.cfg2(2048)
    mu = np.abs(w.mu_true) + 0.5
    obs = w.obs - w.mu_true + mu
    s2 = (2.38 / np.sqrt(16 * w.nobs)) ** 2
    ups = [oracle.mwg_update(2, list(range(0, 32, 2)), sigma=s2 * np.eye(16), prior=L.PRIOR_PRODUCT,
                             factors=[(N_, 6, 1.0, 3.0), (G_, 10, 2.0, 2.0)]),
           oracle.mwg_update(2, list(range(1, 32, 2)), sigma=s2 * np.eye(16), prior=L.PRIOR_STANDARD,
                             factors=[(E_, 1, 2.0, 0.0)] * 16)]
    steps = full_steps(120, 2)
    th0 = np.tile(mu, (2048, 1))
    eng, st, h = run_both(oracle, 32, 2048, 120, ups, mu, np.eye(32), obs, steps, w.seed, ll_mode=ll_mode,
                          theta0=th0)
    assert "mwg_wide_kernel<D=32" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 2)


def test_d32_correlated_joint_proposal_and_target(oracle):
    """A dense Σ at D = 32 for both the GaussianRandomWalk proposal and GsnTargetLaw
    (random_walk.jl:145-171, gsn_target.jl:15-29): rows a5/a10 at the headline D."""
    rng = np.random.default_rng(32)
    B = rng.standard_normal((32, 32))
    S = B @ B.T / 32 + np.eye(32)
    mu = rng.standard_normal(32)
    obs = rng.multivariate_normal(mu, S, size=10)
    R = (2.38 ** 2 / (32 * 10)) * S
    ups = [oracle.mwg_update(2, list(range(32)), sigma=R)]
    steps = full_steps(150, 1)
    eng, st, h = run_both(oracle, 32, 4096, 150, ups, mu, S, obs, steps, 77)
    assert "rwm_gsn_chol_kernel<D=32" in eng.kernel_name()  # the fused correlated-Σ kernel
    check(oracle, eng, st, h, steps, ups, 1)
    assert 0.1 < h["acc"][50:].mean() < 0.45
