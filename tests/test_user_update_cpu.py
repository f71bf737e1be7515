"""User-defined updates on the CPU: the test sources compile for gfx950 through
the library's own hiprtc path (no device needed), and the oracle's gcc build of
them drives a correct Metropolis–Hastings chain — the pCN transition density
does not cancel, so a wrong sign or a swapped argument order would bias the
posterior, which here must be N(x̄, Σ/n) (GsnTargetLaw, ImproperPrior)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.kernels import UserUpdate


@pytest.mark.parametrize("name", ["pcn", "lognormal_walk"])
def test_user_update_sources_compile_for_gfx950(oracle, name):
    _, src = oracle.user_update(name)
    for D in (3, 16, 32):
        L.check_user_update(src, D)


def test_a_broken_update_source_reports_the_compiler_log():
    with pytest.raises(L.EMCMCError) as e:
        L.check_user_update("EMCMC_USER_PROPOSAL { theta_prop[0] = nope; }\nEMCMC_USER_LTD { return 0.0; }", 2)
    assert e.value.status == L.INVALID_ARG and "nope" in str(e.value)


def test_pcn_samples_the_gaussian_posterior(oracle):
    """8192 chains × 1500 pCN steps (ρ = 0.7, centred at 0, so far from x̄: the
    transition density terms carry the correction): posterior mean x̄ and
    variance 1/n per coordinate within Monte Carlo error."""
    D, C, M, n = 3, 8192, 1500, 10
    rng = np.random.default_rng(5)
    mu = np.array([1.0, -0.5, 2.0])
    obs = mu + rng.normal(size=(n, D))
    fns, _ = oracle.user_update("pcn")
    ups = [oracle.mwg_update(oracle.KIND_USER, range(D), params=[0.7, 0.5, 0.0, 0.0, 0.0])]
    st = oracle.MWGState(np.zeros((C, D)), mu, ups)
    oracle.run_mwg(st, ups, seed=21, t_sigma=np.eye(D), obs=obs, steps=[(i, 1) for i in range(1, M + 1)],
                   nthreads=8, history=False, user_upd=fns)
    xb = obs.mean(0)
    m, v = st.theta.mean(0), st.theta.var(0)
    assert np.all(np.abs(m - xb) < 5 * np.sqrt(1.0 / n / C) * 3), (m, xb)
    assert np.all(np.abs(v - 1.0 / n) < 0.15 / n), v
    assert 0.02 < st.nacc[0].mean() / M < 0.9


def test_user_update_mirror_type():
    u = UserUpdate("EMCMC_USER_PROPOSAL {} EMCMC_USER_LTD { return 0.0; }", [1, 3], params=[0.5])
    assert u.coords == [1, 3] and u.invcoords == {1: 1, 3: 2}
