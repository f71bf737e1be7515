"""Shared helpers: run the same workload through the engine (GPU, via the C ABI)
and through the oracle (CPU), with identical seeds and chain ids."""
import numpy as np

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig


def theta0_for(w, C):
    th = np.asarray(w.theta_init, dtype=float)
    return np.ascontiguousarray(np.broadcast_to(th, (C, w.D)) if th.ndim == 1 else th[:C])


def run_engine(w, C, S, *, lpc=0, ll_mode=0, hist=L.HIST_FULL, spl=0, chain0=0, theta0=None, M=None,
               iter_first=1, fetch=True, variant=0):
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=M or (iter_first + S - 1), seed=w.seed,
                              first_chain_id=chain0, history_mode=hist, lanes_per_chain=lpc,
                              steps_per_launch=spl, kernel_variant=variant))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs, ll_mode=ll_mode)
    eng.set_state(theta0_for(w, C) if theta0 is None else theta0)
    eng.run_iters(iter_first, S)
    eng.synchronize(allow_faults=True)
    out = {"engine": eng, "kernel": eng.kernel_name()}
    out["theta"], out["ll"] = eng.get_state()
    ra, nacc = eng.get_chain_stats()
    out["ra"], out["nacc"] = ra[0], nacc[0]
    out["faults"] = eng.get_faults()
    if fetch:
        out["acc"] = eng.get_history(L.H_ACCEPT, iter_first, S)[:, 0]
        if hist == L.HIST_FULL:
            out["theta_hist"] = eng.get_history(L.H_STATE, iter_first, S)[:, 0]
            out["prop_hist"] = eng.get_history(L.H_PROPOSAL, iter_first, S)[:, 0]
            out["ll_hist"] = eng.get_history(L.H_LL, iter_first, S)[:, 0]
    return out


def run_oracle(oracle, w, C, S, *, ll_mode=0, chain0=0, theta0=None, iter_first=1, nthreads=8, history=True):
    st = oracle.OracleState(theta0_for(w, C) if theta0 is None else theta0)
    if iter_first != 1:
        st.N = iter_first
    h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=iter_first,
                       nsteps=S, chain0=chain0, ll_mode=ll_mode, nthreads=nthreads, history=history)
    h["state"] = st
    return h


def assert_bitwise(eng, orc, full=True):
    st = orc["state"]
    assert np.array_equal(eng["acc"], orc["acc"]), \
        f"accept streams differ in {(eng['acc'] != orc['acc']).any(axis=0).sum()} chains"
    assert np.array_equal(eng["theta"], st.theta)
    assert np.array_equal(eng["ll"], st.ll)
    assert np.array_equal(eng["ra"], st.ra)
    assert np.array_equal(eng["nacc"], st.nacc.astype(np.uint64))
    if full:
        assert np.array_equal(eng["ll_hist"], orc["ll"])
        assert np.array_equal(eng["theta_hist"], orc["theta"])
        assert np.array_equal(eng["prop_hist"], orc["prop"])
