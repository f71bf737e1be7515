"""Debug: cfg4 (mix + Haario + chain moments) parity vs oracle at several chain counts."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))
import numpy as np
from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig
from oracle import oracle as O

S = int(sys.argv[1]) if len(sys.argv) > 1 else 400
for C in [int(x) for x in sys.argv[2:]] or [1024, 16384, 131072]:
    w = W.cfg4(C, k=200)
    eng = Engine(EngineConfig(dim=w.D, num_chains=C, num_mcmc_steps=S, seed=w.seed, steps_per_launch=100))
    eng.add_gaussian_rw_mix_update(np.arange(w.D), w.rw_sigma, w.sigma_b, lam=w.lam, haario_k=w.haario_k)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, w.D)))
    eng.run_iters(1, 100); eng.run_iters(101, S - 100)
    eng.synchronize(allow_faults=True)
    acc = eng.get_history(L.H_ACCEPT, 1, S)[:, 0]
    mean, cov = eng.get_chain_moments()
    faults = eng.get_faults()
    print(f"C={C}: faulted {np.count_nonzero(faults)}", flush=True)
    for c in sorted(set([0, 1, C - 1] + list(np.random.default_rng(1).choice(C, 3, replace=False)))):
        st = O.MixState(np.zeros((1, w.D)), sigma_b=w.sigma_b)
        h = O.run_mix(st, seed=w.seed, sigma_a=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=S,
                      lam=w.lam, haario_k=w.haario_k, chain0=int(c))
        bad = np.nonzero(acc[:, c] != h["acc"][:, 0])[0]
        hth = eng.get_history(L.H_STATE, 1, S)[:, 0, c] if C <= 16384 else None
        bth = np.nonzero(np.any(hth != h["theta"][:, 0], axis=1))[0] if hth is not None else []
        print(f"  chain {c}: first acc mismatch {bad[:3]}, first theta mismatch {bth[:3]}, mean eq "
              f"{np.array_equal(mean[c], st.mean[0])}, cov eq {np.array_equal(cov[c], st.cov[0])}, "
              f"maxdiff cov {np.max(np.abs(cov[c]-st.cov[0])):.3e} faults gpu {faults[c]} orc {st.faults[0]}", flush=True)
    eng.close()
