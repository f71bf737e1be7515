"""Row f4 on the GPU: history rings on device (emcmc_config.history_ring) and
asynchronous, thinned streaming to pinned host memory (emcmc_stream_history),
against the oracle's full histories, bit for bit — on the fused, the general
schedule (Metropolis-within-Gibbs) and the mix paths."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _fused(D, C, M, R, seed):
    w = W.cfg2(C, D=D)
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=seed, history_ring=R, steps_per_launch=7))
    eng.add_gaussian_rw_update(range(D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, D)))
    return eng, w


def test_ring_stream_thinned_matches_oracle(oracle):
    """M = 120 iterations through a 16-iteration ring, run in chunks of 10; each
    chunk is streamed right after it is enqueued (state every iteration, ll every
    3rd, accept bits), and the next chunk is enqueued without waiting."""
    D, C, M, R, seed = 8, 300, 120, 16, 77
    eng, w = _fused(D, C, M, R, seed)
    outs = []
    for i0 in range(1, M + 1, 10):
        eng.run_iters(i0, 10)
        outs.append((i0, eng.stream_history(L.H_STATE, i0, 10), eng.stream_history(L.H_LL, i0, 4, thin=3),
                     eng.stream_history(L.H_ACCEPT, i0, 10)))
    eng.synchronize()
    eng.stream_wait()
    st = oracle.OracleState(np.zeros((C, D)))
    h = oracle.run_gsn(st, seed=seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=M,
                       nthreads=8)
    for i0, th, ll, acc in outs:
        assert np.array_equal(th[:, 0], h["theta"][i0 - 1:i0 + 9])
        assert np.array_equal(ll[:, 0], h["ll"][i0 - 1:i0 + 9:3])
        bits = np.unpackbits(acc[:, 0].view(np.uint8), axis=-1, bitorder="little")[:, :C].astype(bool)
        assert np.array_equal(bits, h["acc"][i0 - 1:i0 + 9])
    # the ring keeps the last R iterations; older ones are gone
    assert np.array_equal(eng.get_history(L.H_STATE, M - R + 1, R)[:, 0], h["theta"][M - R:])
    with pytest.raises(L.EMCMCError) as e:
        eng.get_history(L.H_STATE, M - R, 1)
    assert e.value.status == L.STATE_ERROR
    th, _ = eng.get_state()
    assert np.array_equal(th, st.theta)


def test_stream_before_overwrite_is_ordered(oracle):
    """Stream iterations 1..16 of a 16-iteration ring, then enqueue 17..64 at once:
    the copy finishes before those slots are overwritten."""
    D, C, M, R, seed = 4, 256, 64, 16, 5
    eng, w = _fused(D, C, M, R, seed)
    eng.run_iters(1, 16)
    th = eng.stream_history(L.H_PROPOSAL, 1, 16)
    eng.run_iters(17, 48)
    eng.stream_wait()
    eng.synchronize()
    st = oracle.OracleState(np.zeros((C, D)))
    h = oracle.run_gsn(st, seed=seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=M,
                       nthreads=8)
    assert np.array_equal(th[:, 0], h["prop"][:16])


def test_ring_on_mwg_and_mix_paths(oracle):
    w = W.ref_test()
    ups = [oracle.mwg_update(1, [0], eps=[0.5]), oracle.mwg_update(1, [1], eps=[0.5])]
    C, M, R = 200, 50, 8
    eng = Engine(EngineConfig(dim=2, num_chains=C, num_mcmc_steps=M, seed=w.seed, history_ring=R, steps_per_launch=5))
    for u in ups:
        eng.add_uniform_rw_update(u["coords"], u["eps"])
    eng.set_gsn_target([1.0, 2.0], w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, 2)))
    steps = [(i, p) for i in range(1, M + 1) for p in (1, 2)]
    eng.run(steps[:60])
    a = eng.stream_history(L.H_STATE, 23, 8)
    eng.run(steps[60:])
    eng.stream_wait()
    st = oracle.MWGState(np.zeros((C, 2)), [1.0, 2.0], ups)
    h = oracle.run_mwg(st, ups, seed=w.seed, t_sigma=w.t_sigma, obs=w.obs, steps=steps, nthreads=8)
    assert np.array_equal(a.reshape(8 * 2, C, 2), h["theta"][44:60])
    assert np.array_equal(eng.get_history(L.H_LL, M - R + 1, R).reshape(R * 2, C), h["ll"][-2 * R:])
    # mix path
    D = 8
    w2 = W.cfg2(C, D=D)
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=M, seed=3, history_ring=R))
    eng.add_gaussian_rw_mix_update(range(D), w2.rw_sigma, w2.rw_sigma, lam=0.5, haario_k=20)
    eng.set_gsn_target(w2.mu_true, w2.t_sigma, w2.obs)
    eng.set_state(np.zeros((C, D)))
    eng.run_iters(1, M)
    eng.synchronize(allow_faults=True)  # k = 20 < D·… : some chains' Σ_B is not positive definite
    st = oracle.MixState(np.zeros((C, D)), sigma_b=w2.rw_sigma)
    h = oracle.run_mix(st, seed=3, sigma_a=w2.rw_sigma, t_sigma=w2.t_sigma, obs=w2.obs, iter0=1, nsteps=M,
                       haario_k=20, nthreads=8)
    assert np.array_equal(eng.get_history(L.H_STATE, M - R + 1, R)[:, 0], h["theta"][M - R:])
    assert np.array_equal(eng.get_state()[0], st.theta)
    assert np.array_equal(eng.get_faults(), st.faults)
