#!/usr/bin/env python3
"""Throughput of the general schedule kernel (mwg_gsn_kernel / mwg_wide_kernel,
including the run-time-compiled user-law variants) on a few workloads; one JSON
line each.  Kernel time from the engine's HIP events (emcmc_get_timing);
"update_steps_per_s" counts (chain, update) steps, i.e. a P-update iteration
counts P.  Run under rocprofv3 --kernel-trace --stats for the per-kernel view."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "extensiblemcmc.jl_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
from extensible_mcmc import _lib as L  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402
from extensible_mcmc.engine import Engine, EngineConfig  # noqa: E402


def timed(eng, steps, reps=3):
    eng.run(steps[: len(steps) // 10])  # warm-up (first launch also compiles any run-time kernel)
    eng.synchronize(allow_faults=True)
    eng.set_timing(True)
    eng.get_timing(reset=True)
    best = None
    for _ in range(reps):
        eng.run(steps)
        eng.synchronize(allow_faults=True)
        ms, n, b = eng.get_timing(reset=True)
        best = ms if best is None else min(best, ms)
    return best, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--haario-chains", type=int, default=131072)
    ap.add_argument("--haario-iters", type=int, default=400)
    ap.add_argument("--only", default="", help="comma-separated workload names (default: all)")
    ap.add_argument("--variant", type=int, default=0, help="emcmc_config.kernel_variant (EMCMC_VARIANT_* A/B flags)")
    ap.add_argument("--inproc", action="store_true",
                    help="run every selected workload in this process (default: one child process each)")
    ap.add_argument("--child-timeout", type=float, default=300.0, help="seconds per workload process")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))
    names = [n for n in WORKLOADS if not only or n in only]
    if not a.inproc and len(names) > 1:
        return run_isolated(names, a)
    C, M = a.chains, a.iters
    w = W.cfg2(8)
    out = []

    def want(name):
        return not only or name in only

    def report(name, eng, P, ms, nbytes, C=C, M=M, extra=None):
        n = C * M * P
        out.append({"workload": name, "kernel": eng.kernel_name(), "chains": C, "iters": M, "updates": P,
                    "ms": ms, "update_steps_per_s": n / (ms / 1e3), "GBps_algorithmic": nbytes / (ms / 1e3) / 1e9,
                    **(extra or {})})
        print(json.dumps(out[-1]), flush=True)

    # (1) D = 32, two GaussianRandomWalk blocks of 16 coordinates (Metropolis-within-Gibbs)
    if want("mwg_d32_two_blocks"):
        mwg_two_blocks(C, M, w, report)
    if want("mwg_d32_two_blocks_wide"):
        mwg_two_blocks(C, M, w, report, L.VARIANT_NO_BLOCK, "_wide")
    for nm, variant in (("mwg_d64_two_blocks", a.variant), ("mwg_d64_two_blocks_wide", L.VARIANT_NO_BLOCK)):
        if want(nm):
            mwg_d64(nm, C, M, report, variant)
    if want("dense_d32_joint"):
        dense_joint(C, M, w, report)
    if want("user_student_t_d4"):
        user_student_t(C, M, report)
    # (4) the round-3 verdict's correlated Haario case and its general-kernel route
    for name, variant in (("haario_dense_d32", 0), ("haario_dense_d32_general", L.VARIANT_NO_MIX_CHOL)):
        if want(name):
            haario_dense(name, variant, a.haario_chains, a.haario_iters, report)
    if want("mala_gsn_d32"):
        mala_gsn(C, M, report, a.variant)
    if want("pcn_user_d32"):
        pcn_user(C, M, report, a.variant)
    # (5) one random-walk update over all 32 coordinates with a prior / positivity flags: the
    # fused diagonal kernel with the prior compiled in where the prior is a Product of univariates
    # or one MvNormal, else mwg_rw_block_kernel; the "_block" twins force the schedule kernel, "_wide" the wide one
    for name in ("rw_product_normal_d32", "rw_standard_mvnormal_d32", "unif_pos_d32", "rw_standard_mvnormal_d64",
                 "gauss_pos_d32"):
        for suffix, variant in (("", a.variant), ("_block", L.VARIANT_NO_FUSED_PRIOR),
                                ("_wide", L.VARIANT_NO_BLOCK | L.VARIANT_NO_FUSED_PRIOR)):
            if want(name + suffix) or (not only and suffix == ""):
                rw_prior(name, suffix, C, M, report, variant)
    if want("rw_standard_mvnormal_d32_lpc4"):  # four lanes per chain instead of auto's two
        rw_prior("rw_standard_mvnormal_d32", "_lpc4", C, M, report, a.variant, lanes=4)


# every workload, in the order one run measures them
WORKLOADS = ["mwg_d32_two_blocks", "mwg_d32_two_blocks_wide", "mwg_d64_two_blocks", "mwg_d64_two_blocks_wide",
             "dense_d32_joint", "dense_d32_joint_suffstat", "user_student_t_d4", "haario_dense_d32",
             "haario_dense_d32_general", "mala_gsn_d32", "pcn_user_d32", "rw_product_normal_d32",
             "rw_product_normal_d32_block", "rw_product_normal_d32_wide", "rw_standard_mvnormal_d32",
             "rw_standard_mvnormal_d32_block", "rw_standard_mvnormal_d32_wide", "unif_pos_d32", "unif_pos_d32_block", "unif_pos_d32_wide",
             "rw_standard_mvnormal_d32_lpc4", "rw_standard_mvnormal_d64", "rw_standard_mvnormal_d64_wide",
             "gauss_pos_d32", "gauss_pos_d32_wide"]


def run_isolated(names, a):
    """One child process per workload (each measured with a fresh allocator, fresh streams and
    only its own code objects loaded), under a time limit; a child that fails ends the run."""
    import subprocess
    fwd = ["--chains", str(a.chains), "--iters", str(a.iters), "--haario-chains", str(a.haario_chains),
           "--haario-iters", str(a.haario_iters), "--variant", str(a.variant), "--inproc"]
    for n in names:
        only = "dense_d32_joint" if n == "dense_d32_joint_suffstat" else n  # one function measures both
        if n == "dense_d32_joint_suffstat" and "dense_d32_joint" in names:
            continue
        r = subprocess.run([sys.executable, "-u", __file__, "--only", only] + fwd, timeout=a.child_timeout)
        if r.returncode != 0:
            print(f"bench_general: workload {n} exited with {r.returncode}", file=sys.stderr, flush=True)
            return r.returncode
    return 0


def corr_d32(seed=32, D=32, nobs=10):
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((D, D))
    ts = B @ B.T / D + np.eye(D)
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, ts, size=nobs)
    return mu, ts, obs


def haario_dense(name, variant, C, M, report):
    """GaussianRandomWalkMix(Σ_A dense, Σ_B, λ = 0.3) + HaarioTypeAdaptation(k = 100) on
    GsnTargetLaw(μ, BBᵀ/32 + I), 10 observations, per-observation likelihood; the kernel
    time covers step + moments (+ readjust) launch groups."""
    D = 32
    mu, ts, obs = corr_d32()
    sa = 0.2 * (2.38 ** 2 / (D * 10)) * ts
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=3 * M, seed=321, kernel_variant=variant))
    eng.add_gaussian_rw_mix_update(np.arange(D), sa, 0.5 * sa, lam=0.3, haario_k=100)
    eng.set_gsn_target(mu, ts, obs)
    eng.set_state(np.tile(obs.mean(0), (C, 1)))
    eng.run([(i, 1) for i in range(1, M // 10 + 1)])  # warm-up (first launch compiles a run-time kernel)
    eng.synchronize(allow_faults=True)
    eng.set_timing(True)
    eng.get_timing(reset=True)
    it0 = M // 10 + 1
    eng.run([(i, 1) for i in range(it0, it0 + M)])
    eng.synchronize(allow_faults=True)
    ms, n, b = eng.get_timing(reset=True)
    faults = int(np.count_nonzero(eng.get_faults() & L.FAULT_POSDEF))
    report(name, eng, 1, ms, b, C=C, M=M, extra={"posdef_faulted_chains": faults, "readjusts_in_window": M // 100})
    eng.close()


def mala_gsn(C, M, report, variant=0):
    """MALA (ϵ = 0.05) on GsnTargetLaw(μ, BBᵀ/32 + I) at D = 32 (general kernel, the target's
    built-in gradient)."""
    D = 32
    mu, ts, obs = corr_d32(7)
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=2 * M, seed=5, kernel_variant=variant))
    eng.add_mala_update(np.arange(D), 0.05)
    eng.set_gsn_target(mu, ts, obs)
    eng.set_state(np.tile(obs.mean(0), (C, 1)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("mala_gsn_d32", eng, 1, ms, b)
    eng.close()


def pcn_user(C, M, report, variant=0):
    """The pCN user update (tests/user_updates/pcn.c, ρ = 0.9, σ = 0.3, centred at x̄) at D = 32
    on the correlated GsnTargetLaw (general kernel, run-time compiled)."""
    D = 32
    mu, ts, obs = corr_d32(9)
    src = (ROOT / "tests" / "user_updates" / "pcn.c").read_text()
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=2 * M, seed=6, kernel_variant=variant))
    eng.add_user_update(np.arange(D), src, params=np.concatenate([[0.9, 0.3], obs.mean(0)]))
    eng.set_gsn_target(mu, ts, obs)
    eng.set_state(np.tile(obs.mean(0), (C, 1)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("pcn_user_d32", eng, 1, ms, b)
    eng.close()


def rw_prior(name, suffix, C, M, report, variant=0, lanes=0):
    """One joint update over D = 32 coordinates on cfg 2's target (10 observations, per
    observation likelihood, full histories), VERDICT r5 next-step 2's shapes:
      rw_product_normal_d32     GaussianRandomWalk(σ²I) + ProductPrior([Product(32 × Normal)])
      rw_standard_mvnormal_d32  GaussianRandomWalk(σ²I) + StandardPrior(MvNormal(μ0, Σ0)), Σ0 dense
      unif_pos_d32              UniformRandomWalk(ϵ) with positivity flags on every coordinate
      gauss_pos_d32             GaussianRandomWalk(σ²I) with positivity flags on every coordinate
    and rw_standard_mvnormal_d64, the MvNormal shape over D = 64 on the 64-dimensional target."""
    D = 64 if name.endswith("_d64") else 32
    w = W.cfg2(8, D=D)
    shift = 4.0 if name in ("unif_pos_d32", "gauss_pos_d32") else 0.0
    mu = np.asarray(w.mu_true) + shift
    obs = np.asarray(w.obs) - np.asarray(w.mu_true) + mu
    s2 = (2.38 / np.sqrt(D * 10)) ** 2
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed, kernel_variant=variant,
                              lanes_per_chain=lanes))
    if name == "rw_product_normal_d32":
        eng.add_gaussian_rw_update(np.arange(D), s2 * np.eye(D), prior=L.PRIOR_PRODUCT,
                                   prior_factors=[(L.DIST_PRODUCT, D, [(L.DIST_NORMAL, 0.0, 3.0)] * D)])
    elif name.startswith("rw_standard_mvnormal"):
        B = np.random.default_rng(9).standard_normal((D, D))
        eng.add_gaussian_rw_update(np.arange(D), s2 * np.eye(D), prior=L.PRIOR_STANDARD,
                                   prior_factors=[(L.DIST_MVNORMAL, D, np.zeros(D), B @ B.T / D + np.eye(D))])
    elif name == "gauss_pos_d32":
        eng.add_gaussian_rw_update(np.arange(D), 0.05 * s2 * np.eye(D), pos=np.ones(D))
    else:
        eng.add_uniform_rw_update(np.arange(D), 0.06, pos=np.ones(D))
    eng.set_gsn_target(mu, np.eye(D), obs)
    eng.set_state(np.tile(mu, (C, 1)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report(name + suffix, eng, 1, ms, b)
    eng.close()


def mwg_d64(name, C, M, report, variant=0):
    """D = 64 as two GaussianRandomWalk blocks of 32 coordinates (P = 2), the first with a
    ProductPrior of Normals, on a 64-dimensional Gaussian target (10 observations)."""
    D = 64
    w = W.cfg2(8, D=D)
    s2 = (2.38 / np.sqrt(32 * 10)) ** 2
    eng = Engine(EngineConfig(dim=D, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed, kernel_variant=variant))
    eng.add_gaussian_rw_update(np.arange(32), s2 * np.eye(32), prior=L.PRIOR_PRODUCT,
                               prior_factors=[(L.DIST_PRODUCT, 32, [(L.DIST_NORMAL, 0.0, 4.0)] * 32)])
    eng.add_gaussian_rw_update(np.arange(32, 64), s2 * np.eye(32))
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.tile(w.mu_true, (C, 1)))
    steps = [(i, p) for i in range(1, M + 1) for p in (1, 2)]
    ms, b = timed(eng, steps, reps=3)
    report(name, eng, 2, ms, b)
    eng.close()


def mwg_two_blocks(C, M, w, report, variant=0, suffix=""):
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed, kernel_variant=variant))
    for blk in (range(0, 16), range(16, 32)):
        eng.add_gaussian_rw_update(np.array(blk), np.asarray(w.rw_sigma)[:16, :16] * 2.0)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((C, 32)))
    steps = [(i, p) for i in range(1, 2 * M + 1) for p in (1, 2)]
    ms, b = timed(eng, steps[: 2 * M], reps=3)
    report("mwg_d32_two_blocks" + suffix, eng, 2, ms, b)
    eng.close()


def dense_joint(C, M, w, report):
    # (2) D = 32, one joint update with correlated proposal and target Σ
    rng = np.random.default_rng(5)
    A = rng.standard_normal((32, 32))
    St = A @ A.T / 32 + np.eye(32)
    Sr = 0.01 * (np.eye(32) + 0.2 * np.ones((32, 32)))
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(32), Sr)
    eng.set_gsn_target(w.mu_true, St, w.obs)
    eng.set_state(np.zeros((C, 32)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("dense_d32_joint", eng, 1, ms, b)
    eng.close()
    # (2b) the same with the sufficient-statistic likelihood (one solve per step)
    eng = Engine(EngineConfig(dim=32, num_chains=C, num_mcmc_steps=2 * M, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(32), Sr)
    eng.set_gsn_target(w.mu_true, St, w.obs, ll_mode=L.LL_SUFFSTAT)
    eng.set_state(np.zeros((C, 32)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("dense_d32_joint_suffstat", eng, 1, ms, b)
    eng.close()


def user_student_t(C, M, report):
    # (3) user law: student-t regression, D = 4, 50 observations (run-time compiled)
    import user_target_cases as U
    case = U.student_t()
    src = (ROOT / "tests" / "user_targets" / f"{case.name}.c").read_text()
    eng = Engine(EngineConfig(dim=case.D, num_chains=2 * C, num_mcmc_steps=2 * M, seed=case.seed))
    eng.add_gaussian_rw_update(np.arange(case.D), 0.01 * np.eye(case.D))
    eng.set_user_target(src, obs=case.obs, params=case.params, theta0=case.theta0)
    eng.set_state(np.zeros((2 * C, case.D)))
    ms, b = timed(eng, [(i, 1) for i in range(1, M + 1)], reps=3)
    report("user_student_t_d4", eng, 1, ms, b, C=2 * C)
    eng.close()


if __name__ == "__main__":
    sys.exit(main() or 0)
