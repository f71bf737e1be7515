"""Drive every oracle entry point on small problems — run by
tests/test_oracle_sanitized.py in a child process that preloads the ASan/UBSan
runtimes and loads oracle/lib/liboracle_san.so (EMCMC_ORACLE_LIB)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "tests", ROOT / "extensiblemcmc.jl_amd"):
    sys.path.insert(0, str(p))

from oracle import oracle as O  # noqa: E402
import user_target_cases as U  # noqa: E402

rng = np.random.default_rng(0)
# fused path: dense D=2 (reference test), diagonal D=32 both ll modes
for D, dense in ((2, True), (32, False)):
    S = np.array([[1.0, 0.5], [0.5, 1.0]]) if dense else np.eye(D)
    obs = rng.normal(size=(10, D))
    for ll_mode in (0, 1):
        st = O.OracleState(np.zeros((7, D)))
        O.run_gsn(st, seed=3, rw_sigma=0.2 * np.eye(D), t_sigma=S, obs=obs, iter0=1, nsteps=25, ll_mode=ll_mode)
# general kernel: priors, pos flags, per-coordinate adaptation, D = 64 block tree
adapt = {"k": 5, "target": 0.234, "scale": [0.1, 0.2], "min": [1e-12, 1e-3], "max": [10.0, 1.0],
         "offset": [1.0, 2.0]}
ups = [O.mwg_update(1, [0, 1], eps=[0.3, 0.2], adapt=adapt, pos=[True, False]),
       O.mwg_update(2, [2, 3], sigma=[[0.1, 0.02], [0.02, 0.1]], pos=[False, True], prior=O.PRIOR_PRODUCT,
                    factors=[(32, 2, [(1, 0.0, 2.0), (4, 2.0, 1.0)])]),
       O.mwg_update(2, [4, 5, 6], sigma=0.1 * np.eye(3), prior=O.PRIOR_PRODUCT,
                    factors=[(1, 1, 0.0, 2.0), (33, 2, [0.0, 0.0], [[1.0, 0.3], [0.3, 1.0]])])]
st = O.MWGState(np.full((5, 7), 0.5), np.zeros(7), ups)
O.run_mwg(st, ups, seed=4, t_sigma=np.eye(7), obs=rng.normal(size=(6, 7)), steps=[(i, p) for i in range(1, 31) for p in (1, 2, 3)])
ups64 = [O.mwg_update(2, range(0, 40), sigma=0.01 * np.eye(40)), O.mwg_update(2, range(40, 64), sigma=0.01 * np.eye(24))]
st = O.MWGState(np.zeros((3, 64)), np.zeros(64), ups64)
O.run_mwg(st, ups64, seed=5, t_sigma=np.eye(64), obs=rng.normal(size=(4, 64)), steps=[(i, p) for i in range(1, 11) for p in (1, 2)])
# a user law
case = U.student_t()
fn, _ = O.user_loglik(case.name)
ups = [O.mwg_update(2, range(case.D), sigma=0.01 * np.eye(case.D))]
st = O.MWGState(np.zeros((4, case.D)), case.theta0, ups)
O.run_mwg(st, ups, seed=6, t_sigma=None, obs=case.obs, steps=[(i, 1) for i in range(1, 21)], user_ll=fn,
          user_params=case.params)
# mix + Haario (a readjust inside the run)
D = 8
st = O.MixState(np.zeros((4, D)), sigma_b=0.05 * np.eye(D))
O.run_mix(st, seed=7, sigma_a=0.02 * np.eye(D), t_sigma=np.eye(D), obs=rng.normal(size=(10, D)), iter0=1, nsteps=30,
          lam=0.5, haario_k=10)
# MALA on a small logistic problem
D, N = 16, 50
X = rng.normal(size=(N, D))
y = (rng.random(N) < 0.5).astype(float)
st = O.MALAState(np.zeros((3, D)), X, y)
O.run_mala(st, seed=8, eps=0.05, X=X, y=y, iter0=1, nsteps=10)
print("sanitized oracle run: ok", O.LIB_PATH.name)
