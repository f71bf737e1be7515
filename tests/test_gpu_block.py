"""mwg_block_kernel on the GPU (VERDICT r4 missing item 2): one MALA update or one
user update (updates.jl:42-93, 129-133; run.jl:110, 259) over all 17 ≤ D ≤ 64
coordinates with every per-chain vector in registers, against the oracle
(orc_run_mwg kinds 4 and 5 — the same restatement the general kernel is checked
against), bit for bit: accept streams, θ / θ° / ll histories, sub_ws°.ll, rolling
acceptance.  D = 32 MALA on GsnTargetLaw is compiled ahead of time; other D, the
pCN user update and a user law go through hiprtc (prebuilt into the on-disk cache
by scripts/prebuild_rtc.py)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig
from extensible_mcmc.schedule import MCMCSchedule
from test_gpu_mwg import check, full_steps

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def corr_problem(D, seed, nobs=10, dense=True):
    """GsnTargetLaw(μ, BBᵀ/D + I) (or a diagonal Σ) with nobs observations; the bench's
    correlated D = 32 target (scripts/bench_general.py corr_d32)."""
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((D, D))
    ts = B @ B.T / D + np.eye(D) if dense else np.diag(rng.uniform(0.5, 2.0, size=D))
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, ts, size=nobs)
    return mu, ts, obs


def run_block(oracle, D, C, M, ups, mu, ts, obs, steps, seed, ll_mode=L.LL_PER_OBS, hist=L.HIST_FULL, spl=0,
              user_src=None):
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist,
                              steps_per_launch=spl))
    u = ups[0]
    if u["kind"] == oracle.KIND_MALA:
        eng.add_mala_update(u["coords"], u["eps"][0])
    else:
        eng.add_user_update(u["coords"], user_src, u["params"])
    eng.set_gsn_target(mu, ts, obs, ll_mode=ll_mode)
    th0 = np.ascontiguousarray(np.broadcast_to(obs.mean(0), (C, D)))
    eng.set_state(th0)
    eng.run(steps)
    st = oracle.MWGState(np.array(th0), mu, ups)
    kw = {}
    if user_src is not None:
        kw["user_upd"] = oracle.user_update("pcn")[0]
    h = oracle.run_mwg(st, ups, seed=seed, t_sigma=ts, obs=obs, steps=steps, ll_mode=ll_mode, nthreads=8, **kw)
    return eng, st, h


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("hist", [L.HIST_FULL, L.HIST_ACCEPT_ONLY])
def test_mala_d32_dense_target(oracle, ll_mode, hist):
    """The bench shape: MALA(ϵ = 0.05) on GsnTargetLaw(μ, BBᵀ/32 + I), 10 observations,
    launches of 23 steps (∇ℓ recomputed at each launch's first step, carried after)."""
    D, C, M = 32, 2048, 60
    mu, ts, obs = corr_problem(D, 7)
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[0.05])]
    steps = full_steps(M, 1)
    eng, st, h = run_block(oracle, D, C, M, ups, mu, ts, obs, steps, 5, ll_mode=ll_mode, hist=hist, spl=23)
    assert eng.kernel_name().startswith("mwg_block_kernel<D=32"), eng.kernel_name()
    assert "[hiprtc]" not in eng.kernel_name()  # ahead of time
    check(oracle, eng, st, h, steps, ups, 1, full=hist == L.HIST_FULL)
    assert 0.2 < h["acc"][1:].mean()


def test_mala_d32_diagonal_target_with_a_gapped_schedule(oracle):
    """A diagonal Σ_t and iterations 11:17 excluded (the accept draws of 2m, 2m+1 share a
    Philox block: a gap must not reuse a stale one)."""
    D, C, M = 32, 1024, 50
    mu, ts, obs = corr_problem(D, 8, dense=False)
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[0.08])]
    steps = [(s.mcmciter, s.pidx) for s in MCMCSchedule(M, 1, [(1, range(11, 18))])]
    eng, st, h = run_block(oracle, D, C, M, ups, mu, ts, obs, steps, 6)
    assert "DIAG_T" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


@pytest.mark.parametrize("D", [20, 40])
def test_mala_at_other_d_compiled_at_run_time(oracle, D):
    C, M = 1024, 30
    mu, ts, obs = corr_problem(D, D, nobs=6)
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[0.04])]
    steps = full_steps(M, 1)
    eng, st, h = run_block(oracle, D, C, M, ups, mu, ts, obs, steps, 7)
    assert eng.kernel_name().startswith(f"mwg_block_kernel<D={D}") and "[hiprtc]" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


def test_pcn_user_update_d32(oracle):
    """The bench's pCN user update (ρ = 0.9, σ = 0.3, centred at x̄) over all 32 coordinates
    of the correlated target, on the block kernel."""
    D, C, M = 32, 2048, 60
    mu, ts, obs = corr_problem(D, 9)
    _, src = oracle.user_update("pcn")
    ups = [oracle.mwg_update(oracle.KIND_USER, range(D), params=[0.9, 0.3] + list(obs.mean(0)))]
    steps = full_steps(M, 1)
    eng, st, h = run_block(oracle, D, C, M, ups, mu, ts, obs, steps, 8, spl=37, user_src=src)
    assert eng.kernel_name().startswith("mwg_block_kernel<D=32") and "UserUpdate" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)
    assert 0.05 < h["acc"][1:].mean() < 0.95


def test_mala_on_a_user_law_d20(oracle):
    """The user logistic-regression law with its EMCMC_USER_GRAD, one MALA update over all
    20 coordinates (block kernel, TGT = the user's law)."""
    rng = np.random.default_rng(21)
    D, n, C, M = 20, 80, 2048, 40
    X = np.column_stack([np.ones(n), rng.normal(size=(n, D - 1))])
    beta = rng.normal(scale=0.3, size=D)
    y = (rng.uniform(size=n) < 1.0 / (1.0 + np.exp(-(X @ beta)))).astype(float)
    obs = np.column_stack([X, y])
    fn, src = oracle.user_loglik("logistic_regression")
    gfn = oracle.user_grad("logistic_regression")
    ups = [oracle.mwg_update(oracle.KIND_MALA, range(D), eps=[0.06])]
    steps = full_steps(M, 1)
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=41))
    eng.add_mala_update(range(D), 0.06)
    eng.set_user_target(src, obs=obs, theta0=np.zeros(D))
    eng.set_state(np.zeros((C, D)))
    eng.run(steps)
    assert eng.kernel_name().startswith("mwg_block_kernel<D=20") and "UserTarget" in eng.kernel_name()
    st = oracle.MWGState(np.zeros((C, D)), np.zeros(D), ups)
    h = oracle.run_mwg(st, ups, seed=41, t_sigma=None, obs=obs, steps=steps, nthreads=8, user_ll=fn, user_grad=gfn)
    check(oracle, eng, st, h, steps, ups, 1)
