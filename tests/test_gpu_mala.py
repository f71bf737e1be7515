"""Row f2 on the GPU (BASELINE cfg 3): mala_logistic_kernel (fp64 MFMA for
η = Xθ° and ∇ℓ = Xᵀr) against the oracle (orc_run_mala), bit for bit — accept
stream, θ, θ°, ll, rolling acceptance — through the C ABI.  The oracle restates
the kernel's evaluation order; v_mfma_f64_16x16x4f64 is an fma chain over k
(scripts/ubench/mfma_f64_probe.hip)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _problem(N, D, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D)) / np.sqrt(D)
    tt = rng.standard_normal(D)
    y = (rng.random(N) < 1 / (1 + np.exp(-X @ tt))).astype(float)
    return X, y


def _engine(X, y, C, M, eps, seed, hist=L.HIST_FULL, theta0=None):
    D = X.shape[1]
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_mode=hist))
    eng.add_mala_update(range(D), eps)
    eng.set_logistic_target(X, y)
    eng.set_state(np.zeros((C, D)) if theta0 is None else theta0)
    return eng


def _check(eng, st, hists, iters, full):
    eng.synchronize(allow_faults=True)
    th, ll = eng.get_state()
    assert np.array_equal(th, st.theta)
    assert np.array_equal(ll, st.ll)
    ra, nacc = eng.get_chain_stats()
    assert np.array_equal(ra[0], st.ra)
    assert np.array_equal(nacc[0], st.nacc)
    assert np.array_equal(eng.get_faults(), st.faults)
    i0, n = iters[0], iters[-1] - iters[0] + 1
    rows = np.asarray(iters) - i0
    assert np.array_equal(eng.get_history(L.H_ACCEPT, i0, n)[rows, 0], np.concatenate([h["acc"] for h in hists]))
    if full:
        for which, key in ((L.H_STATE, "theta"), (L.H_PROPOSAL, "prop"), (L.H_LL, "ll")):
            got = eng.get_history(which, i0, n)[rows, 0]
            assert np.array_equal(got, np.concatenate([h[key] for h in hists])), key


@pytest.mark.parametrize("D,N,C,eps,hist", [
    (16, 1000, 200, 0.08, L.HIST_FULL),     # N and C off the 64-row / 64-chain tiles
    (32, 1234, 130, 0.12, L.HIST_ACCEPT_ONLY),
    (48, 640, 64, 0.2, L.HIST_FULL),
    (64, 3000, 256, 0.25, L.HIST_FULL),
])
def test_mala_matches_oracle(oracle, D, N, C, eps, hist):
    X, y = _problem(N, D)
    M = 60
    eng = _engine(X, y, C, M, eps, seed=11, hist=hist)
    eng.run_iters(1, M)
    assert "mala_logistic_kernel<D=%d" % D in eng.kernel_name()
    st = oracle.MALAState(np.zeros((C, D)), X, y, nthreads=8)
    h = oracle.run_mala(st, seed=11, eps=eps, X=X, y=y, iter0=1, nsteps=M, nthreads=8)
    assert 0.2 < h["acc"].mean() <= 1.0
    _check(eng, st, [h], list(range(1, M + 1)), hist == L.HIST_FULL)


def test_mala_split_calls_and_gap(oracle):
    """Three emcmc_run calls and a schedule gap (iterations 21:25 skipped):
    the carried ∇ℓ is reused across calls, rolling_ar restarts after the gap."""
    X, y = _problem(900, 16)
    C, eps = 100, 0.1
    eng = _engine(X, y, C, 60, eps, seed=4)
    iters = list(range(1, 21)) + list(range(26, 51))
    for a, b in ((0, 7), (7, 30), (30, len(iters))):
        eng.run([(i, 1) for i in iters[a:b]])
    st = oracle.MALAState(np.zeros((C, 16)), X, y, nthreads=8)
    hs = [oracle.run_mala(st, seed=4, eps=eps, X=X, y=y, iter0=1, nsteps=20, nthreads=8),
          oracle.run_mala(st, seed=4, eps=eps, X=X, y=y, iter0=26, nsteps=25, nthreads=8)]
    _check(eng, st, hs, iters, True)


def test_cfg3_shape_bitwise(oracle):
    """The cfg 3 shape (N = 100,000, D = 64) on 256 chains for 4 steps."""
    w = W.cfg3(256)
    eng = _engine(w.X, w.y, 256, 4, w.eps, seed=w.seed)
    eng.run_iters(1, 4)
    st = oracle.MALAState(np.zeros((256, 64)), w.X, w.y, nthreads=8)
    h = oracle.run_mala(st, seed=w.seed, eps=w.eps, X=w.X, y=w.y, iter0=1, nsteps=4, nthreads=8)
    _check(eng, st, [h], [1, 2, 3, 4], True)


def test_mala_rejects_other_shapes():
    X, y = _problem(100, 20)
    eng = Engine(EngineConfig(dim=20, num_chains=64, num_mcmc_steps=10))
    eng.add_mala_update(range(20), 0.1)
    with pytest.raises(L.EMCMCError) as e:
        eng.set_logistic_target(X, y)
    assert e.value.status == L.UNSUPPORTED_PLUGIN
    X, y = _problem(100, 16)
    eng = Engine(EngineConfig(dim=16, num_chains=64, num_mcmc_steps=10))
    eng.add_gaussian_rw_update(range(16), 0.01 * np.eye(16))
    with pytest.raises(L.EMCMCError) as e:
        eng.set_logistic_target(X, y)
    assert e.value.status == L.UNSUPPORTED_PLUGIN


def test_cfg3_grid_on_sampled_chains(oracle):
    """The real cfg 3 grid (32,768 chains, N = 1e5, D = 64: 512 workgroups re-reading X
    from L2/MALL) for 3 steps; 8 chains across the grid — first and last workgroups,
    different XCDs — replayed on the oracle, bit for bit: accept stream, θ / θ° / ll
    histories and the final state."""
    w = W.cfg3()
    C, M = w.num_chains, 3
    eng = _engine(w.X, w.y, C, M, w.eps, w.seed)
    eng.run_iters(1, M)
    eng.synchronize()
    th, ll = eng.get_state()
    acc = eng.get_history(L.H_ACCEPT, 1, M)[:, 0]
    hth = eng.get_history_chains(L.H_STATE, 1, M, 0, C)
    picks = [0, 1, 63, 64, 4097, 16383, 20000, C - 1]
    for c in picks:
        st = oracle.MALAState(np.zeros((1, w.D)), w.X, w.y, nthreads=16)
        h = oracle.run_mala(st, seed=w.seed, eps=w.eps, X=w.X, y=w.y, iter0=1, nsteps=M, chain0=c, nthreads=16)
        assert np.array_equal(acc[:, c], h["acc"][:, 0]), c
        assert np.array_equal(th[c], st.theta[0]) and ll[c] == st.ll[0], c
        assert np.array_equal(hth[:, 0, c], h["theta"][:, 0]), c
