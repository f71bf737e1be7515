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
P_, MV_ = L.DIST_PRODUCT, L.DIST_MVNORMAL


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
        # StandardPrior(Product([…])): a univariate StandardPrior has no scalar logpdf on θ::Vector
        pk, fs = [L.PRIOR_STANDARD, L.PRIOR_STANDARD], [[(P_, 1, [(U_, -3.0, 3.0)])], [(P_, 1, [(E_, 2.0, 0.0)])]]
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
    """A ProductPrior([Product([Uniform(−0.3, 0.3), Uniform(1.7, 2.3)])], [2]) with proposals
    ~10× wider than the support: most draws are resampled (normal indices (r << 17) | j),
    every accepted state stays inside, and the streams match the oracle bitwise."""
    w = W.ref_test()
    fs = [(P_, 2, [(U_, -0.3, 0.3), (U_, 1.7, 2.3)])]
    ups = [oracle.mwg_update(2, [0, 1], sigma=[[4.0, 0.0], [0.0, 4.0]], prior=L.PRIOR_PRODUCT, factors=fs)]
    steps = full_steps(200, 1)
    th0 = np.tile([0.0, 2.0], (512, 1))
    eng, st, h = run_both(oracle, 2, 512, 200, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed, theta0=th0)
    check(oracle, eng, st, h, steps, ups, 1)
    assert np.all(np.abs(h["prop"][..., 0]) <= 0.3) and np.all(np.abs(h["prop"][..., 1] - 2.0) <= 0.3)
    assert not np.any(st.faults & L.FAULT_PRIOR_RESAMPLES)


@pytest.mark.parametrize("variant", [0, L.VARIANT_NO_BLOCK])
@pytest.mark.parametrize("ll_mode", [0, 1])
def test_d32_two_blocks_with_priors(oracle, ll_mode, variant):
    """Metropolis-within-Gibbs at the headline D = 32: two GaussianRandomWalk blocks of
    16 coordinates, a ProductPrior of Product(Normal)/Product(Gamma) factors on one and a
    StandardPrior(Product(Exponential)) on the other (so a Gaussian target at μ* > 0 keeps mass
    in the support) — on the compiled-schedule block kernel (round 6) and on the wide kernel."""
    w = W.cfg2(2048)
    mu = np.abs(w.mu_true) + 0.5
    obs = w.obs - w.mu_true + mu
    s2 = (2.38 / np.sqrt(16 * w.nobs)) ** 2
    ups = [oracle.mwg_update(2, list(range(0, 32, 2)), sigma=s2 * np.eye(16), prior=L.PRIOR_PRODUCT,
                             factors=[(P_, 6, [(N_, 1.0, 3.0)] * 6), (P_, 10, [(G_, 2.0, 2.0)] * 10)]),
           oracle.mwg_update(2, list(range(1, 32, 2)), sigma=s2 * np.eye(16), prior=L.PRIOR_STANDARD,
                             factors=[(P_, 16, [(E_, 2.0, 0.0)] * 16)])]
    steps = full_steps(120, 2)
    th0 = np.tile(mu, (2048, 1))
    eng, st, h = run_both(oracle, 32, 2048, 120, ups, mu, np.eye(32), obs, steps, w.seed, ll_mode=ll_mode,
                          theta0=th0, variant=variant)
    assert ("mwg_wide_kernel<D=32" if variant else "mwg_rw_block_kernel<D=32") in eng.kernel_name()
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


def test_product_prior_dims1_factors_read_theta1(oracle):
    """ProductPrior([Normal(1, .5), Gamma(4, .5)], [1, 1]) on a 2-coordinate GaussianRandomWalk:
    both factors read θ[1] (priors.jl:68-70), θ[2] is unconstrained; bitwise against the
    oracle, and the mirror's logpdf of every θ history equals that reading."""
    from extensible_mcmc import Gamma, Normal, ProductPrior
    from extensible_mcmc.kernels import prior_to_device

    w = W.ref_test()
    pr = ProductPrior([Normal(1.0, 0.5), Gamma(4.0, 0.5)], [1, 1])
    kind, fs = prior_to_device(pr, 2)
    ups = [oracle.mwg_update(2, [0, 1], sigma=[[0.2, 0.05], [0.05, 0.3]], prior=kind, factors=fs)]
    steps = full_steps(250, 1)
    th0 = np.tile([1.0, 2.0], (777, 1))
    eng, st, h = run_both(oracle, 2, 777, 250, ups, [1.0, 2.0], w.t_sigma, w.obs, steps, w.seed, theta0=th0)
    check(oracle, eng, st, h, steps, ups, 1)
    # the Gamma factor on θ[1] keeps θ[1] > 0; θ[2] takes negative values freely (it is not read)
    assert np.all(h["theta"][..., 0] > 0)
    assert 0.05 < h["acc"].mean() < 0.95


def test_product_prior_with_mvnormal_and_all_families(oracle):
    """A UniformRandomWalk block of 10 positivity-restricted coordinates under
    ProductPrior([Exponential(2), Product([LogNormal, Gamma, Beta, InverseGamma, …]), …])
    and a GaussianRandomWalk block of 4 under ProductPrior([Normal, MvNormal(3)], [1, 3]):
    every family and the MvNormal forward substitution, bitwise against the oracle."""
    rng = np.random.default_rng(41)
    D, C, M = 14, 1000, 150
    comps = [(L.DIST_LOGNORMAL, 0.0, 0.8), (G_, 3.0, 0.4), (L.DIST_BETA, 2.0, 3.0), (L.DIST_INVERSE_GAMMA, 3.0, 2.0),
             (L.DIST_CAUCHY, 1.0, 0.5), (L.DIST_LAPLACE, 1.0, 0.7), (L.DIST_TDIST, 3.5, 0.0), (N_, 1.0, 1.0),
             (U_, 0.0, 4.0)]
    B = rng.standard_normal((3, 3))
    S3 = B @ B.T / 3 + 0.5 * np.eye(3)
    fa = [(E_, 1, 2.0, 0.0), (P_, 9, comps)]
    fb = [(N_, 1, 0.0, 2.0), (MV_, 3, np.array([0.5, -0.5, 0.0]), S3)]
    ups = [oracle.mwg_update(1, range(10), eps=[0.15] * 10, pos=[True] * 10, prior=L.PRIOR_PRODUCT, factors=fa),
           oracle.mwg_update(2, range(10, 14), sigma=0.05 * np.eye(4), prior=L.PRIOR_PRODUCT, factors=fb)]
    mu = np.concatenate([[0.5, 1.0, 1.0, 0.4, 0.8, 1.0, 1.0, 1.0, 1.0, 1.0], rng.standard_normal(4)])
    obs = mu + 0.5 * rng.standard_normal((5, D))
    th0 = np.tile(np.concatenate([[0.5, 1.0, 1.0, 0.4, 0.8, 1.0, 1.0, 1.0, 1.0, 1.0], np.zeros(4)]), (C, 1))
    steps = full_steps(M, 2)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, 4.0 * np.eye(D), obs, steps, 4242, theta0=th0)
    check(oracle, eng, st, h, steps, ups, 2)
    assert 0.05 < h["acc"].mean() < 0.95


@pytest.mark.parametrize("case", ["univariate_dims3", "mvnormal_dims1", "standard_univariate", "past_the_end"])
def test_prior_pairings_without_a_reference_value_are_refused(case):
    """The pairings the reference raises on (MethodError / BoundsError) are refused by the
    engine."""
    from extensible_mcmc.engine import Engine, EngineConfig

    eng = Engine(EngineConfig(dim=3, num_chains=64, num_mcmc_steps=4, seed=1, device=0))
    want = L.UNSUPPORTED_PLUGIN
    try:
        if case == "univariate_dims3":
            fs, kind = [(N_, 3, 0.0, 1.0)], L.PRIOR_PRODUCT
        elif case == "mvnormal_dims1":
            fs, kind = [(MV_, 1, [0.0], [[1.0]]), (P_, 2, [(N_, 0.0, 1.0)] * 2)], L.PRIOR_PRODUCT
        elif case == "standard_univariate":
            fs, kind = [(N_, 1, 0.0, 1.0)], L.PRIOR_STANDARD
        else:
            fs, kind, want = [(N_, 1, 0.0, 1.0), (P_, 3, [(N_, 0.0, 1.0)] * 3)], L.PRIOR_PRODUCT, L.INVALID_ARG
        with pytest.raises(L.EMCMCError) as e:
            eng.add_gaussian_rw_update(np.arange(3), 0.1 * np.eye(3), prior=kind, prior_factors=fs)
            eng.set_gsn_target(np.zeros(3), np.eye(3), np.zeros((2, 3)))
            eng.set_state(np.zeros((64, 3)))
            eng.run_iters(1, 2)
        assert e.value.status == want
    finally:
        eng.close()


def test_chain_moments_with_a_prior_run_on_the_general_kernel(oracle):
    """emcmc_config.chain_moments with a prior on the joint update (no prior term in the
    fused cfg 4 kernels): the general kernel keeps GenericChainStats mean/cov, bitwise."""
    from extensible_mcmc.engine import Engine, EngineConfig

    rng = np.random.default_rng(8)
    D, C, M = 3, 512, 80
    mu = rng.normal(size=D)
    obs = mu + rng.normal(size=(6, D))
    fs = [(P_, 3, [(N_, 0.0, 3.0)] * 3)]
    ups = [oracle.mwg_update(2, range(D), sigma=0.1 * np.eye(D), prior=L.PRIOR_PRODUCT, factors=fs)]
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=3, chain_moments=True))
    eng.add_gaussian_rw_update(np.arange(D), 0.1 * np.eye(D), prior=L.PRIOR_PRODUCT, prior_factors=fs)
    eng.set_gsn_target(mu, np.eye(D), obs)
    eng.set_state(np.tile(mu, (C, 1)))
    eng.run_iters(1, M)
    assert eng.kernel_name().startswith("mwg_gsn_kernel")
    st = oracle.MWGState(np.tile(mu, (C, 1)), mu, ups, chain_moments=True)
    oracle.run_mwg(st, ups, seed=3, t_sigma=np.eye(D), obs=obs, steps=full_steps(M, 1), nthreads=8, history=False)
    eng.synchronize()
    th, _ = eng.get_state()
    m, v = eng.get_chain_moments()
    assert np.array_equal(th, st.theta)
    assert np.array_equal(m, st.smean) and np.array_equal(v, st.scov)
