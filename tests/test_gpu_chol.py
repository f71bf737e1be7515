"""rwm_gsn_chol_kernel: a correlated Σ at D ≥ 16 for the GaussianRandomWalk
proposal and/or GsnTargetLaw (random_walk.jl:145-171, gsn_target.jl:15-29;
rows a5/a10 at the headline D), factors read through the scalar cache with
column-sweep forward substitutions.  Bar: the whole accept stream, θ, θ°, ll
histories and the carried state bit for bit against the oracle's row-order
formulas (oracle/emcmc_oracle.c sqmahal / run_chain), for both likelihood modes,
full and accept-only histories, ragged chain counts and launch splits."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W

from helpers import assert_bitwise, run_engine, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _corr(D, seed, dense_rw=True, dense_t=True, nobs=10):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((D, D))
    S = A @ A.T / D + np.eye(D) if dense_t else np.diag(rng.uniform(0.5, 2.0, D))
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, S, size=nobs)
    B = rng.standard_normal((D, D))
    R = (2.38 ** 2 / (D * nobs)) * ((B @ B.T / D + np.eye(D)) if dense_rw else np.diag(rng.uniform(0.5, 2.0, D)))
    return W.GsnWorkload(f"chol_d{D}", D, 0, mu, S, R, obs, mu.copy(), seed=1000 + seed)


@pytest.mark.parametrize("D", [16, 24, 32])
@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
def test_chol_kernel_correlated_bitwise(oracle, D, ll_mode):
    w = _corr(D, D)
    e = run_engine(w, 2048, 120, ll_mode=ll_mode)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},")
    o = run_oracle(oracle, w, 2048, 120, ll_mode=ll_mode)
    assert_bitwise(e, o)
    assert 0.05 < e["acc"][20:].mean() < 0.8


@pytest.mark.parametrize("dense_rw,dense_t", [(True, False), (False, True)])
def test_chol_kernel_one_side_correlated(oracle, dense_rw, dense_t):
    """Dense proposal with a diagonal target and the reverse: the diagonal factor
    goes through the same column sweeps (zero off-diagonals, exact)."""
    w = _corr(32, 7, dense_rw, dense_t)
    e = run_engine(w, 1000, 90)  # 1000 chains: a partial last wave
    assert "chol" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 1000, 90))


def test_chol_kernel_accept_only_and_launch_splits(oracle):
    w = _corr(32, 11)
    o = run_oracle(oracle, w, 777, 70)
    for spl in (1, 9, 64):
        e = run_engine(w, 777, 70, hist=L.HIST_ACCEPT_ONLY, spl=spl)
        assert "chol" in e["kernel"] and "ACCEPT_ONLY" in e["kernel"]
        assert_bitwise(e, o, full=False)


def test_chol_kernel_overdispersed_start_and_shards(oracle):
    """Chains start far from the mode (rejections dominate early, θ° far in the
    tails) and a second shard keyed at chain id 4096 reproduces the oracle."""
    w = _corr(32, 13)
    th0 = w.mu_true + 3.0 * np.random.default_rng(3).standard_normal((512, 32))
    e = run_engine(w, 512, 60, chain0=4096, theta0=th0)
    assert_bitwise(e, run_oracle(oracle, w, 512, 60, chain0=4096, theta0=th0))


@pytest.mark.parametrize("D,ll_mode", [(9, L.LL_PER_OBS), (12, L.LL_SUFFSTAT), (20, L.LL_PER_OBS),
                                       (40, L.LL_SUFFSTAT), (48, L.LL_PER_OBS), (64, L.LL_PER_OBS)])
def test_chol_kernel_compiled_at_run_time(oracle, D, ll_mode):
    """A correlated Σ at a D without an ahead-of-time instantiation: the same
    rwm_gsn_chol_kernel compiled with hiprtc (chunks of 16/8/4/2/1 doubles as D
    allows), bitwise against the oracle — where round 2 ran the general kernel."""
    w = _corr(D, 100 + D)
    e = run_engine(w, 1536, 60, ll_mode=ll_mode)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},") and "[hiprtc]" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 1536, 60, ll_mode=ll_mode))
    assert 0.02 < e["acc"][10:].mean() < 0.9


def test_chol_rtc_equals_general_kernel(oracle):
    """EMCMC_VARIANT_NO_RTC_CHOL keeps the round-2 route (the general kernel); both
    routes give the same bits at D = 20."""
    w = _corr(20, 5)
    a = run_engine(w, 512, 40)
    b = run_engine(w, 512, 40, variant=L.VARIANT_NO_RTC_CHOL)
    assert "chol" in a["kernel"] and "mwg" in b["kernel"]
    for k in ("acc", "theta", "ll", "ra", "nacc", "theta_hist", "prop_hist", "ll_hist"):
        assert np.array_equal(a[k], b[k]), k


def test_chol_rtc_accept_only_and_launch_splits(oracle):
    """The run-time compiled kernel (D = 20) with accept-only histories, a ragged chain
    count and launches of 1, 7 and 64 steps: the same bits as one full-history launch."""
    w = _corr(20, 17)
    o = run_oracle(oracle, w, 999, 50)
    for spl in (1, 7, 64):
        e = run_engine(w, 999, 50, hist=L.HIST_ACCEPT_ONLY, spl=spl)
        assert "[hiprtc]" in e["kernel"] and "ACCEPT_ONLY" in e["kernel"]
        assert_bitwise(e, o, full=False)


def test_chol_rtc_compile_limit_routes_to_general_kernel(oracle):
    """D = 27 (odd: one-double scalar-load chunks, 405 per sweep) is above the run-time
    chol kernel's compile budget: the general kernel runs it, bitwise."""
    w = _corr(27, 27)
    e = run_engine(w, 256, 12)
    assert "mwg" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 256, 12))
