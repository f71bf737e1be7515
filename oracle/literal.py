"""Literal numpy restatement of the reference MH loop — TEST INFRASTRUCTURE ONLY.

Pure-Python loop over steps (small cases only).  It restates the reference
formulas as written, with numpy/LAPACK arithmetic (no canonical summation
order), and takes its random variates from the shared counter-based stream via
oracle.step_variates.  It checks the C oracle's canonical-order arithmetic
within fp64 tolerance and bit-for-bit on the accept/reject stream.

Reference lines restated (under /root/reference/src):
  run.jl:101-112   update_workspaces!: θ copy; ll carried; −Inf before step 1
  random_walk.jl:145-151  θ° = rand(MvNormal(θ, Σ))  = θ + chol(Σ).L z
  random_walk.jl:161-171  logpdf(rw, θ, θ°) = logpdf(MvNormal(θ, Σ), θ°) + logJ (logJ = −0.0, pos all false)
  gsn_target.jl:23-29     ll = 0.0; for obs: ll += logpdf(P.P, obs)
  run.jl:271-278   llr = ll° − ll + ltd(θ°→θ) − ltd(θ→θ°) + lp(θ°) − lp(θ); accept = E > −llr
  run.jl:312-335   θ ← θ° and ll_hist ← ll° on accept
  chain_statistics.jl:53-65  rolling acceptance
"""
from __future__ import annotations

import numpy as np

try:
    from scipy.linalg import solve_triangular
except Exception:  # pragma: no cover
    solve_triangular = None

from . import oracle as _oracle  # type: ignore  # noqa: E402

LOG2PI = float(np.log(2 * np.pi))


def mvnormal_logpdf(x, mu, L):
    """Distributions: mvnormal_c0(d) − sqmahal(d, x)/2 with L = cholesky(Σ).L."""
    D = L.shape[0]
    r = np.asarray(x, dtype=float) - np.asarray(mu, dtype=float)
    y = solve_triangular(L, r, lower=True) if solve_triangular else np.linalg.solve(L, r)
    logdet = 2.0 * np.sum(np.log(np.diag(L)))
    return -(D * LOG2PI + logdet) / 2.0 - float(np.dot(y, y)) / 2.0


def run_chain(seed, chain, theta0, rw_sigma, t_sigma, obs, nsteps, iter0=1, W=100, ll0=-np.inf, ll_mode=0):
    Lrw = np.linalg.cholesky(np.asarray(rw_sigma, dtype=float))
    Lt = np.linalg.cholesky(np.asarray(t_sigma, dtype=float))
    obs = np.asarray(obs, dtype=float)
    D = Lrw.shape[0]
    th = np.array(theta0, dtype=float)
    ll = float(ll0)
    ra = 0.0
    acc_hist = {}
    out = {"theta": [], "prop": [], "ll": [], "acc": [], "ra": []}
    N = 1
    for s in range(nsteps):
        it = iter0 + s
        z, E, _ = _oracle.step_variates(seed, chain, it, D)
        thp = th + Lrw @ z
        llp = 0.0
        for x in obs:
            llp += mvnormal_logpdf(x, thp, Lt)
        ltd_fwd = mvnormal_logpdf(thp, th, Lrw) + (-0.0)
        ltd_rev = mvnormal_logpdf(th, thp, Lrw) + (-0.0)
        llr = llp - ll + ltd_rev - ltd_fwd + 0.0 - 0.0
        acc = E > -llr
        if acc:
            th = thp
            ll = llp
        acc_hist[it] = acc
        outside = acc_hist.get(it - W, False) if it > W else False
        ra = (ra * W + (int(acc) - int(outside))) / min(W, N)
        N += 1
        out["theta"].append(th.copy())
        out["prop"].append(thp.copy())
        out["ll"].append(ll)
        out["acc"].append(acc)
        out["ra"].append(ra)
    return {k: np.array(v) for k, v in out.items()}
