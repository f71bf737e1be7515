"""mix_chol_kernel: GaussianRandomWalkMix + HaarioTypeAdaptation (and GaussianRandomWalk
with GenericChainStats mean/cov) with a dense Σ_A and a correlated target Σ_t at
D = 16 / 32 on the fused path (random_walk.jl:193-232, adaptation.jl:399-426,
chain_statistics.jl:41-66): L_A and L_t through the scalar cache, each chain's L_B
streamed from HBM, the batched moments and readjust kernels of cfg 4.  Bar: bit for
bit against the oracle's kind-3 restatement (orc_run_mwg, the general kernel's
reference) through readjusts, and equal to the general kernel's own run
(EMCMC_VARIANT_NO_MIX_CHOL)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from test_gpu_mix_general import check_mix, run_both
from test_gpu_mwg import check, full_steps

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def corr_target(D, seed, nobs=10):
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((D, D))
    ts = B @ B.T / D + np.eye(D)
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, ts, size=nobs)
    return mu, ts, obs


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
def test_correlated_haario_d32_fused_through_two_readjusts(oracle, ll_mode):
    """The verdict's case on the fused path: Haario on GsnTargetLaw(μ, BBᵀ/32 + I),
    dense Σ_A, k = 100, 230 steps (two readjusts), bitwise against kind 3."""
    D, C, M, k = 32, 1024, 230, 100
    mu, ts, obs = corr_target(D, 32)
    sa = 0.2 * (2.38 ** 2 / (D * 10)) * ts
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=sa, sigma_b=0.5 * sa, lam=0.3, haario_k=k)]
    steps = full_steps(M, 1)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, ts, obs, steps, 321, theta0=obs.mean(0), ll_mode=ll_mode)
    assert eng.kernel_name().startswith("mix_chol_kernel<D=32,"), eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups)
    assert st.M[0] == M % k
    posdef = (st.faults & L.FAULT_POSDEF) != 0
    assert posdef.mean() < 0.05
    assert 0.3 < h["acc"][1:].mean() < 0.9


@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_correlated_haario_d16_launch_splits(oracle, hist):
    """D = 16, a ragged chain count, launches of 37 steps that do not line up with the
    readjust period (k = 60), both history modes."""
    D, C, M, k = 16, 777, 200, 60
    mu, ts, obs = corr_target(D, 16, nobs=7)
    sa = 0.3 * (2.38 ** 2 / (D * 7)) * ts
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=sa, sigma_b=sa, lam=0.5, haario_k=k)]
    steps = full_steps(M, 1)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, ts, obs, steps, 77, theta0=mu, hist=hist, spl=37)
    assert eng.kernel_name().startswith("mix_chol_kernel<D=16,")
    check(oracle, eng, st, h, steps, ups, 1, full=hist == L.HIST_FULL)
    check_mix(oracle, eng, st, ups)


def test_dense_gaussian_rw_with_chain_moments_d32(oracle):
    """GaussianRandomWalk(dense Σ) + GenericChainStats mean/cov (emcmc_config.chain_moments)
    on a correlated target: the MIX = false instantiation."""
    D, C, M = 32, 640, 120
    mu, ts, obs = corr_target(D, 5)
    sa = 0.5 * (2.38 ** 2 / (D * 10)) * ts
    ups = [oracle.mwg_update(2, range(D), sigma=sa)]
    steps = full_steps(M, 1)
    eng, st, h = run_both(oracle, D, C, M, ups, mu, ts, obs, steps, 9, theta0=mu, chain_moments=True)
    assert eng.kernel_name().startswith("mix_chol_kernel<D=32,") and "GSN_MOMENTS" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    check_mix(oracle, eng, st, ups, chain_moments=True)


def test_fused_equals_general_kernel(oracle):
    """EMCMC_VARIANT_NO_MIX_CHOL keeps the general kernel; both routes give the same
    bits, L_B and Haario moments included."""
    D, C, M, k = 32, 512, 150, 50
    mu, ts, obs = corr_target(D, 8)
    sa = 0.2 * (2.38 ** 2 / (D * 10)) * ts
    ups = [oracle.mwg_update(oracle.KIND_MIX, range(D), sigma=sa, sigma_b=0.7 * sa, lam=0.4, haario_k=k)]
    steps = full_steps(M, 1)
    out = []
    for variant in (0, L.VARIANT_NO_MIX_CHOL):
        from extensible_mcmc.engine import Engine, EngineConfig

        eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=11, kernel_variant=variant))
        eng.add_gaussian_rw_mix_update(np.arange(D), sa, 0.7 * sa, lam=0.4, haario_k=k)
        eng.set_gsn_target(mu, ts, obs)
        eng.set_state(np.tile(mu, (C, 1)))
        eng.run(steps)
        th, ll = eng.get_state()
        acc = eng.get_history(L.H_ACCEPT, 1, M)
        hth = eng.get_history(L.H_STATE, 1, M)
        lb, m = eng.get_mix_state(1)
        hm, hc = eng.get_adaptation_moments(1)
        out.append((eng.kernel_name(), th, ll, acc, hth, lb, m, hm, hc))
        eng.close()
    assert out[0][0].startswith("mix_chol_kernel") and "mwg" in out[1][0]
    for a, b in zip(out[0][1:], out[1][1:]):
        assert np.array_equal(a, b)
