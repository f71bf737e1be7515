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


def run_mwg_chain(seed, chain, theta0, mu0, updates, t_sigma, obs, steps, W=100, chain_moments=False):
    """Literal single-chain restatement of the P-update loop (see
    oracle/emcmc_oracle.c orc_run_mwg for the reference lines): plain Python
    floats and numpy/LAPACK for the MvNormal logpdf.  GaussianRandomWalkMix
    updates (kind 3) with HaarioTypeAdaptation register the global θ view of
    their coordinates after every step, in place through remove/reimpose
    (adaptation.jl:406-414), and readjust Σ_B = 2.38²/n·cov on their own turn."""
    Lt = np.linalg.cholesky(np.asarray(t_sigma, dtype=float))
    obs = np.asarray(obs, dtype=float)
    th = np.array(theta0, dtype=float)
    mp = np.array(mu0, dtype=float)           # P°.θ[1:d], starts at the target's μ
    P = len(updates)
    eps = [list(u["eps"]) if u["eps"] is not None else None for u in updates]
    prop_c, acc_c = [0] * P, [0] * P
    ll = -np.inf
    N = 1
    ra = {}                                    # (iter, p) → rolling_ar value
    acc_hist = {}
    out = {"theta": [], "prop": [], "ll": [], "acc": [], "ra": [], "eps": []}
    SB = [np.asarray(u["sigma_b"], dtype=float) if u["kind"] == 3 else None for u in updates]
    hmean = [np.zeros(len(u["coords"])) for u in updates]
    hcov = [np.zeros((len(u["coords"]),) * 2) for u in updates]
    M = [0] * P
    smean, scov = np.zeros(th.size), np.zeros((th.size, th.size))
    for it, pidx in steps:
        p = pidx - 1
        u = updates[p]
        cs = u["coords"]
        tl = th[cs].copy()
        ta = None
        if u["kind"] == 1:                     # UniformRandomWalk (random_walk.jl:63-94)
            pos = [bool(x) for x in u["pos"]] if u.get("pos") is not None else [False] * len(cs)
            tp = np.empty_like(tl)
            for j in range(len(cs)):
                a, b = -eps[p][j], eps[p][j]
                U = a + (b - a) * _oracle.uniform01(seed, chain, it, p, j)
                tp[j] = tl[j] * (np.exp(U) * pos[j] + 1.0 * (not pos[j])) + U * (not pos[j])
            # logpdf(rw, θ, θ°) = mapreduce(i -> pos[i] ? -log(2ϵ_i) - log(θ°_i) : 0.0, +, 1:n)
            fwd = [(-np.log(2.0 * eps[p][j]) - np.log(tp[j])) if pos[j] else 0.0 for j in range(len(cs))]
            rev = [(-np.log(2.0 * eps[p][j]) - np.log(tl[j])) if pos[j] else 0.0 for j in range(len(cs))]
            ltd_fwd, ltd_rev = fwd[0], rev[0]
            for j in range(1, len(cs)):
                ltd_fwd, ltd_rev = ltd_fwd + fwd[j], ltd_rev + rev[j]
        elif u["kind"] == 4:                   # MALA (the engine's definition; the reference stubs it)
            # compute_gradients_and_momenta!(__PREVIOUS) (run.jl:110) at P°.θ with coords ← θ:
            # ∇ℓ(μ) = Σ_k Σ⁻¹(x_k − μ); θ° = θ + (ϵ²/2)g + ϵz; MvNormal(·, ϵ²I) both ways
            e = float(u["eps"][0])
            hm = e * e / 2.0
            Le = e * np.eye(len(cs))
            x = mp.copy()
            x[cs] = tl
            g = sum(np.linalg.solve(Lt @ Lt.T, xo - x) for xo in obs)[cs]
            z, _, _ = _oracle.step_variates(seed, chain, it, len(cs), pidx0=p)
            m = tl + hm * g
            tp = m + e * z
            ltd_fwd = mvnormal_logpdf(tp, m, Le)
            ltd_rev = None                     # after set_proposal! (run.jl:259)
        elif u["kind"] == 3:                   # GaussianRandomWalkMix (random_walk.jl:193-232)
            n = len(cs)
            pos = np.array(u["pos"], dtype=bool) if u.get("pos") is not None else np.zeros(n, dtype=bool)
            LA = np.linalg.cholesky(np.asarray(u["sigma"], dtype=float))
            LB = np.linalg.cholesky(SB[p])        # raises LinAlgError ≙ PosDefException
            lam = u["lam"]
            useB = _oracle.pick_uniform(seed, chain, it, p) <= lam   # pick_kernel: rand(Bernoulli(λ))
            Lr = LB if useB else LA
            z, _, _ = _oracle.step_variates(seed, chain, it, n, pidx0=p)
            th_l = tl.copy()                   # state(ws)
            th_l[pos] = np.log(th_l[pos])      # rand(gsn_X, θ): remove_constraints!
            th_o = th_l + Lr @ z
            th_o[pos] = np.exp(th_o[pos])
            th_l[pos] = np.exp(th_l[pos])
            tp = th_o.copy()

            def gsn_logpdf(a, b, Lx):          # logpdf(gsn_X, a, b), mutating a and b (:166-171)
                logJ = -sum(np.log(b[pos]))    # −sum(empty) = −0.0 without positivity flags
                a[pos] = np.log(a[pos])
                b[pos] = np.log(b[pos])
                lp = mvnormal_logpdf(b, a, Lx) + logJ
                a[pos] = np.exp(a[pos])
                b[pos] = np.exp(b[pos])
                return lp

            def mix_logpdf(a, b):              # log((1−λ)e^{lp_A} + λe^{lp_B}) (:229-232)
                lpa = gsn_logpdf(a, b, LA)
                lpb = gsn_logpdf(a, b, LB)
                return np.log((1 - lam) * np.exp(lpa) + lam * np.exp(lpb))
            ltd_rev = mix_logpdf(th_o, th_l)   # __PROPOSAL first (run.jl:271-277)
            ltd_fwd = mix_logpdf(th_l, th_o)
            ta = th_o.copy()
        else:                                  # GaussianRandomWalk
            Lr = np.linalg.cholesky(np.asarray(u["sigma"], dtype=float))
            z, _, _ = _oracle.step_variates(seed, chain, it, len(cs), pidx0=p)
            pos = np.array(u["pos"], dtype=bool) if u.get("pos") is not None else np.zeros(len(cs), dtype=bool)
            if not pos.any():
                tp = tl + Lr @ z
                ltd_fwd = mvnormal_logpdf(tp, tl, Lr)
                ltd_rev = mvnormal_logpdf(tl, tp, Lr)
            else:                              # random_walk.jl:136-171, in-place as written
                th_l = tl.copy()               # state(ws)
                th_l[pos] = np.log(th_l[pos])  # remove_constraints!(rw, θ)
                th_o = th_l + Lr @ z           # rand(MvNormal(θ, Σ))
                th_o[pos] = np.exp(th_o[pos])  # reimpose_constraints!(rw, θ°)
                th_l[pos] = np.exp(th_l[pos])  # reimpose_constraints!(rw, θ)
                tp = th_o.copy()               # state°(ws) as set_proposal! sees it

                def rw_logpdf(a, b):           # logpdf(rw, a, b), mutating a and b
                    logJ = -sum(np.log(b[pos]))
                    a[pos] = np.log(a[pos])
                    b[pos] = np.log(b[pos])
                    lp = mvnormal_logpdf(b, a, Lr) + logJ
                    a[pos] = np.exp(a[pos])
                    b[pos] = np.exp(b[pos])
                    return lp
                ltd_rev = rw_logpdf(th_o, th_l)  # log_transition_density(__PROPOSAL): θ° → θ
                ltd_fwd = rw_logpdf(th_l, th_o)  # log_transition_density(__PREVIOUS): θ → θ°
                ta = th_o.copy()                 # what set_chain_param! copies on accept
        if ta is None:
            ta = tp
        prop = th.copy()
        prop[cs] = tp
        mp[cs] = tp                            # set_parameters!(P°, coords, θ°)
        llp = 0.0
        for x in obs:
            llp += mvnormal_logpdf(x, mp, Lt)
        if u["kind"] == 4:                     # compute_gradients_and_momenta!(__PROPOSAL) at P°.θ
            gp = sum(np.linalg.solve(Lt @ Lt.T, xo - mp) for xo in obs)[cs]
            ltd_rev = mvnormal_logpdf(tl, tp + hm * gp, Le)
        _, E, _ = _oracle.step_variates(seed, chain, it, 1, pidx0=p)
        llr = llp - ll + ltd_rev - ltd_fwd + 0.0 - 0.0
        acc = bool(E > -llr)
        if acc:
            th[cs] = ta
            ll = llp
        acc_hist[(it, p)] = acc
        prev = ra.get((it - 1, p), 0.0) if it > 1 else 0.0
        outside = acc_hist.get((it - W, p), False) if it > W else False
        ra[(it, p)] = (prev * W + (int(acc) - int(outside))) / min(W, N)
        N += 1
        if u["adapt"] is not None:             # AdaptationUnifRW, own turn
            ad = u["adapt"]
            acc_c[p] += int(acc)
            prop_c[p] += 1
            if prop_c[p] >= ad["k"]:
                # compute_δ / compute_ϵ (adaptation.jl:312-329), coordinate by
                # coordinate for the per-coordinate form (scalars broadcast)
                nj = len(eps[p])
                vec = lambda v: [float(v)] * nj if np.ndim(v) == 0 else [float(x) for x in v]  # noqa: E731
                sc, mn, mx, off = vec(ad["scale"]), vec(ad["min"]), vec(ad["max"]), vec(ad["offset"])
                a_r = 0.0 if prop_c[p] == 0 else acc_c[p] / prop_c[p]
                prop_c[p] = acc_c[p] = 0
                eps[p] = [max(min(e + 1.0 * (2 * int(a_r > ad["target"]) - 1) *
                                  (sc[j] / np.sqrt(max(1.0, it / ad["k"] - off[j]))), mx[j]), mn[j])
                          for j, e in enumerate(eps[p])]
        out["theta"].append(th.copy())
        if chain_moments:                      # update_stats! (chain_statistics.jl:46-49), N before += 1
            Nc = N - 1
            old_sum_sq = (Nc - 1) / Nc * scov + np.outer(smean, smean)
            smean = smean * (Nc / (Nc + 1)) + th / (Nc + 1)
            new_sum_sq = old_sum_sq + np.outer(th, th) / Nc
            scov = new_sum_sq - (Nc + 1) / Nc * np.outer(smean, smean)
        for q, v in enumerate(updates):        # update_adaptation! (run.jl:136-178)
            if not v.get("haario_k"):
                continue
            Nh = N - 1
            if q == p:
                M[q] += 1                      # register_only_on_my_turn(Val(true)) (adaptation.jl:401-404)
            cq = v["coords"]
            posq = np.array(v["pos"], dtype=bool) if v.get("pos") is not None else np.zeros(len(cq), dtype=bool)
            x = th[cq]                         # state(global_ws, updt): a view; remove_constraints! on it
            x[posq] = np.log(x[posq])
            old_sum_sq = (Nh - 1) / Nh * hcov[q] + np.outer(hmean[q], hmean[q])
            hmean[q] = hmean[q] * (Nh / (Nh + 1)) + x / (Nh + 1)
            new_sum_sq = old_sum_sq + np.outer(x, x) / Nh
            hcov[q] = new_sum_sq - (Nh + 1) / Nh * np.outer(hmean[q], hmean[q])
            x[posq] = np.exp(x[posq])          # reimpose_constraints!
            th[cq] = x
            if q == p and M[q] >= v["haario_k"]:   # time_to_update → readjust!
                M[q] = 0
                S_new = 2.38 ** 2 / len(cq) * hcov[q]
                try:                           # the reference throws PosDefException at the next
                    np.linalg.cholesky(S_new)  # MvNormal; the engine keeps the factor (fault bit 4)
                    SB[q] = S_new
                except np.linalg.LinAlgError:
                    out.setdefault("posdef_faults", []).append((it, q))
        out["prop"].append(prop)
        out["ll"].append(ll)
        out["acc"].append(acc)
        out["ra"].append(ra[(it, p)])
        out["eps"].append([list(e) if e is not None else None for e in eps])
    out["state"] = th.copy()
    out["smean"], out["scov"] = smean, scov
    out["hmean"], out["hcov"], out["sigma_b"] = hmean, hcov, SB
    return out


def run_mix_chain(seed, chain, theta0, sigma_a, sigma_b, lam, t_sigma, obs, nsteps, haario_k=0, mix=True, W=100):
    """Literal single-chain GaussianRandomWalkMix (+ HaarioTypeAdaptation) and
    GenericChainStats mean/cov (random_walk.jl:193-232, adaptation.jl:372-426,
    chain_statistics.jl:41-66), matrix formulas as written: Cholesky of Σ_A and
    Σ_B at every call (LAPACK), the rank-one recurrence with numpy outer
    products, Σ_B = 2.38²/D·cov at each readjust."""
    SA = np.asarray(sigma_a, dtype=float)
    SB = np.asarray(sigma_b, dtype=float)
    Lt = np.linalg.cholesky(np.asarray(t_sigma, dtype=float))
    obs = np.asarray(obs, dtype=float)
    D = SA.shape[0]
    th = np.array(theta0, dtype=float)
    ll = -np.inf
    ra = 0.0
    acc_hist = {}
    mean = np.zeros(D)
    cov = np.zeros((D, D))
    N, M = 1, 0
    out = {"theta": [], "prop": [], "ll": [], "acc": [], "ra": [], "cov": [], "mean": []}
    for s in range(nsteps):
        it = 1 + s
        LA = np.linalg.cholesky(SA)
        LB = np.linalg.cholesky(SB)            # raises LinAlgError ≙ PosDefException
        useB = mix and _oracle.pick_uniform(seed, chain, it) <= lam
        z, E, _ = _oracle.step_variates(seed, chain, it, D)
        thp = th + (LB if useB else LA) @ z
        if mix:
            def lmix(x, m):
                return np.log((1 - lam) * np.exp(mvnormal_logpdf(x, m, LA) + (-0.0))
                              + lam * np.exp(mvnormal_logpdf(x, m, LB) + (-0.0)))
            ltd_fwd, ltd_rev = lmix(thp, th), lmix(th, thp)
        else:
            ltd_fwd, ltd_rev = mvnormal_logpdf(thp, th, LA), mvnormal_logpdf(th, thp, LA)
        llp = 0.0
        for x in obs:
            llp += mvnormal_logpdf(x, thp, Lt)
        llr = llp - ll + ltd_rev - ltd_fwd + 0.0 - 0.0
        acc = bool(E > -llr)
        if acc:
            th = thp
            ll = llp
        # update_stats!
        old_sum_sq = (N - 1) / N * cov + np.outer(mean, mean)
        mean = mean * (N / (N + 1)) + th / (N + 1)
        new_sum_sq = old_sum_sq + np.outer(th, th) / N
        cov = new_sum_sq - (N + 1) / N * np.outer(mean, mean)
        acc_hist[it] = acc
        outside = acc_hist.get(it - W, False) if it > W else False
        ra = (ra * W + (int(acc) - int(outside))) / min(W, N)
        N += 1
        if haario_k:                           # M += 1 on own turn; readjust at M ≥ k
            M += 1
            if M >= haario_k:
                M = 0
                SB = 2.38 ** 2 / D * cov
        out["theta"].append(th.copy())
        out["prop"].append(thp.copy())
        out["ll"].append(ll)
        out["acc"].append(acc)
        out["ra"].append(ra)
    out["cov"], out["mean"], out["sigma_b"] = cov, mean, SB
    return {k: (np.array(v) if isinstance(v, list) else v) for k, v in out.items()}


def run_mala_chain(seed, chain, theta0, eps, X, y, nsteps, W=100):
    """Literal MALA on the logistic target: numpy matrix-vector products,
    np.logaddexp softplus, MvNormal(m, ϵ²I) logpdf via mvnormal_logpdf."""
    X = np.asarray(X, dtype=float)
    y = np.asarray(y, dtype=float)
    D = X.shape[1]
    h = eps * eps / 2.0
    L = eps * np.eye(D)

    def ell_grad(th):
        eta = X @ th
        ll = float(np.sum(y * eta - np.logaddexp(0.0, eta)))
        sig = 0.5 * (1.0 + np.tanh(0.5 * eta))
        return ll, X.T @ (y - sig)

    th = np.array(theta0, dtype=float)
    _, g = ell_grad(th)
    ll = -np.inf
    ra, N = 0.0, 1
    acc_hist = {}
    out = {"theta": [], "prop": [], "ll": [], "acc": [], "ra": []}
    for s in range(nsteps):
        it = 1 + s
        z, E, _ = _oracle.step_variates(seed, chain, it, D)
        m = th + h * g
        tp = m + eps * z
        llp, gp = ell_grad(tp)
        ltd_fwd = mvnormal_logpdf(tp, m, L)
        ltd_rev = mvnormal_logpdf(th, tp + h * gp, L)
        llr = llp - ll + ltd_rev - ltd_fwd + 0.0 - 0.0
        acc = bool(E > -llr)
        if acc:
            th, ll, g = tp, llp, gp
        acc_hist[it] = acc
        outside = acc_hist.get(it - W, False) if it > W else False
        ra = (ra * W + (int(acc) - int(outside))) / min(W, N)
        N += 1
        out["theta"].append(th.copy())
        out["prop"].append(tp.copy())
        out["ll"].append(ll)
        out["acc"].append(acc)
        out["ra"].append(ra)
    return {k: np.array(v) for k, v in out.items()}
