"""User-defined target laws (row g1) on the CPU: the hiprtc build of each source
for gfx950 (no device needed), the compile-error path, the oracle's gcc build of
the same sources against numpy restatements, and the protocol pin: a user law
that restates GsnTargetLaw gives the oracle's built-in chain bit for bit."""
import numpy as np
import pytest

import user_target_cases as U
from extensible_mcmc import _lib as L


@pytest.mark.parametrize("name,D", [("student_t_regression", 4), ("poisson_regression", 3), ("banana", 2),
                                    ("banana", 24), ("banana", 64), ("gsn_identity", 3), ("gsn_full", 6),
                                    ("gsn_full", 20)])
def test_user_source_compiles_for_gfx950(oracle, name, D):
    _, src = oracle.user_loglik(name)
    L.check_user_target(src, D)  # raises with the hiprtc log on error


def test_user_source_compile_error_is_reported():
    bad = "EMCMC_USER_LOGLIK { return theta[0] + undefined_symbol; }"
    with pytest.raises(L.EMCMCError) as e:
        L.check_user_target(bad, 2)
    assert e.value.status == L.INVALID_ARG
    assert "undefined_symbol" in str(e.value)


def test_gradient_named_only_in_a_comment_is_not_a_gradient():
    """A law that mentions EMCMC_USER_GRAD only in a comment or a string defines no
    gradient: it compiles as a plain law (before, a text search compiled the MALA
    path in and the build failed on an undefined emcmc_user_grad)."""
    src = ("/* no EMCMC_USER_GRAD here */\n// nor EMCMC_USER_GRAD here\n"
           "EMCMC_USER_LOGLIK { const char *s = \"EMCMC_USER_GRAD\"; (void)s; return -0.5 * theta[0] * theta[0]; }")
    L.check_user_target(src, 2)


def test_user_target_rejects_too_large_dim(oracle):
    _, src = oracle.user_loglik("banana")
    with pytest.raises(L.EMCMCError):
        L.check_user_target(src, 65)


@pytest.mark.parametrize("make", [U.student_t, U.poisson, U.banana, U.gsn_identity, U.gsn_full])
def test_oracle_user_loglik_matches_numpy(oracle, make):
    import ctypes as C
    case = make()
    fn, _ = oracle.user_loglik(case.name)
    rng = np.random.default_rng(7)
    obs = np.ascontiguousarray(case.obs, dtype=np.float64)
    prm = np.ascontiguousarray(case.params, dtype=np.float64)
    dp = C.POINTER(C.c_double)
    for _ in range(20):
        th = np.ascontiguousarray(rng.normal(scale=0.5, size=case.D) + case.theta0)
        if case.name == "gsn_full":  # keep Σ positive definite
            d = case.extra["d"]
            th[d:] = (np.eye(d) * 2.0 + 0.1 * rng.normal(size=(d, d))).ravel(order="F")
        got = fn(th.ctypes.data_as(dp), case.D, obs.ctypes.data_as(dp), obs.shape[0], prm.ctypes.data_as(dp))
        want = U.numpy_loglik(case, th)
        assert got == pytest.approx(want, rel=1e-12, abs=1e-12)


def test_gsn_as_user_law_reproduces_builtin_target_bitwise(oracle):
    """Protocol pin: GsnTargetLaw(θ, I) as a user law (tests/user_targets/gsn_identity.c)
    in orc_run_mwg gives the built-in GsnTargetLaw chain, bit for bit."""
    case = U.gsn_identity()
    fn, _ = oracle.user_loglik(case.name)
    C, D, M = 64, case.D, 60
    ups = [oracle.mwg_update(2, range(D), sigma=0.3 * np.eye(D))]
    steps = [(i, 1) for i in range(1, M + 1)]
    runs = []
    for user in (False, True):
        st = oracle.MWGState(np.zeros((C, D)), case.theta0, ups)
        h = oracle.run_mwg(st, ups, seed=case.seed, t_sigma=np.eye(D), obs=case.obs, steps=steps,
                           user_ll=fn if user else None, user_params=case.params if user else None)
        runs.append((st, h))
    (a, ha), (b, hb) = runs
    assert np.array_equal(a.theta, b.theta) and np.array_equal(a.ll, b.ll)
    for k in ("theta", "prop", "ll", "acc"):
        assert np.array_equal(ha[k], hb[k]), k
    assert 0.05 < ha["acc"][1:].mean() < 0.95


def test_full_gsn_law_with_fixed_sigma_is_the_builtin_law(oracle):
    """GsnTargetLaw over θ = [μ; vec Σ] as a user law (tests/user_targets/gsn_full.c),
    updating μ only, gives the built-in GsnTargetLaw(μ, Σ) chain bit for bit (the
    canonical Cholesky, logdet and forward substitution restated in the source)."""
    case = U.gsn_full()
    d = case.extra["d"]
    fn, _ = oracle.user_loglik(case.name)
    C, M = 48, 80
    th0 = np.concatenate([np.zeros(d), case.extra["S"].ravel(order="F")])
    steps = [(i, p) for i in range(1, M + 1) for p in (1, 2)]
    ups = [oracle.mwg_update(2, [0], sigma=[[0.4]]), oracle.mwg_update(1, [1], eps=[0.6])]
    a = oracle.MWGState(np.tile(th0, (C, 1)), th0, ups)
    ha = oracle.run_mwg(a, ups, seed=case.seed, t_sigma=None, obs=case.obs, steps=steps, user_ll=fn,
                        user_params=case.params)
    b = oracle.MWGState(np.zeros((C, d)), case.extra["mu"] * 0 + th0[:d], ups)
    hb = oracle.run_mwg(b, ups, seed=case.seed, t_sigma=case.extra["S"], obs=case.obs, steps=steps)
    assert np.array_equal(a.theta[:, :d], b.theta) and np.array_equal(a.ll, b.ll)
    assert np.array_equal(ha["acc"], hb["acc"]) and np.array_equal(ha["ll"], hb["ll"])
