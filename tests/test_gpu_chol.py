"""rwm_gsn_chol_kernel: a correlated Σ at D ≥ 16 for the GaussianRandomWalk
proposal and/or GsnTargetLaw (random_walk.jl:145-171, gsn_target.jl:15-29;
rows a5/a10 at the headline D), factors read through the scalar cache with
column-sweep forward substitutions.  Bar: the whole accept stream, θ, θ°, ll
histories and the carried state bit for bit against the oracle's row-order
formulas (oracle/emcmc_oracle.c sqmahal / run_chain), for both likelihood modes,
full and accept-only histories, ragged chain counts and launch splits."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W

from helpers import assert_bitwise, run_engine, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def _corr(D, seed, dense_rw=True, dense_t=True, nobs=10):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((D, D))
    S = A @ A.T / D + np.eye(D) if dense_t else np.diag(rng.uniform(0.5, 2.0, D))
    mu = rng.standard_normal(D)
    obs = rng.multivariate_normal(mu, S, size=nobs)
    B = rng.standard_normal((D, D))
    R = (2.38 ** 2 / (D * nobs)) * ((B @ B.T / D + np.eye(D)) if dense_rw else np.diag(rng.uniform(0.5, 2.0, D)))
    return W.GsnWorkload(f"chol_d{D}", D, 0, mu, S, R, obs, mu.copy(), seed=1000 + seed)


@pytest.mark.parametrize("D", [16, 24, 32])
@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
def test_chol_kernel_correlated_bitwise(oracle, D, ll_mode):
    w = _corr(D, D)
    e = run_engine(w, 2048, 120, ll_mode=ll_mode)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},")
    o = run_oracle(oracle, w, 2048, 120, ll_mode=ll_mode)
    assert_bitwise(e, o)
    assert 0.05 < e["acc"][20:].mean() < 0.8


@pytest.mark.parametrize("dense_rw,dense_t", [(True, False), (False, True)])
def test_chol_kernel_one_side_correlated(oracle, dense_rw, dense_t):
    """Dense proposal with a diagonal target and the reverse: the diagonal factor
    goes through the same column sweeps (zero off-diagonals, exact)."""
    w = _corr(32, 7, dense_rw, dense_t)
    e = run_engine(w, 1000, 90)  # 1000 chains: a partial last wave
    assert "chol" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 1000, 90))


def test_chol_kernel_accept_only_and_launch_splits(oracle):
    w = _corr(32, 11)
    o = run_oracle(oracle, w, 777, 70)
    for spl in (1, 9, 64):
        e = run_engine(w, 777, 70, hist=L.HIST_ACCEPT_ONLY, spl=spl)
        assert "chol" in e["kernel"] and "ACCEPT_ONLY" in e["kernel"]
        assert_bitwise(e, o, full=False)


def test_chol_kernel_overdispersed_start_and_shards(oracle):
    """Chains start far from the mode (rejections dominate early, θ° far in the
    tails) and a second shard keyed at chain id 4096 reproduces the oracle."""
    w = _corr(32, 13)
    th0 = w.mu_true + 3.0 * np.random.default_rng(3).standard_normal((512, 32))
    e = run_engine(w, 512, 60, chain0=4096, theta0=th0)
    assert_bitwise(e, run_oracle(oracle, w, 512, 60, chain0=4096, theta0=th0))


@pytest.mark.parametrize("D,ll_mode", [(9, L.LL_PER_OBS), (12, L.LL_SUFFSTAT), (20, L.LL_PER_OBS),
                                       (40, L.LL_SUFFSTAT), (48, L.LL_PER_OBS), (64, L.LL_PER_OBS)])
def test_chol_kernel_compiled_at_run_time(oracle, D, ll_mode):
    """A correlated Σ at a D without an ahead-of-time instantiation: the same
    rwm_gsn_chol_kernel compiled with hiprtc (chunks of 16/8/4/2/1 doubles as D
    allows), bitwise against the oracle — where round 2 ran the general kernel."""
    w = _corr(D, 100 + D)
    e = run_engine(w, 1536, 60, ll_mode=ll_mode)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},") and "[hiprtc]" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 1536, 60, ll_mode=ll_mode))
    assert 0.02 < e["acc"][10:].mean() < 0.9


def test_chol_rtc_equals_general_kernel(oracle):
    """EMCMC_VARIANT_NO_RTC_CHOL keeps the round-2 route (the general kernel); both
    routes give the same bits at D = 20."""
    w = _corr(20, 5)
    a = run_engine(w, 512, 40)
    b = run_engine(w, 512, 40, variant=L.VARIANT_NO_RTC_CHOL)
    assert "chol" in a["kernel"] and "mwg" in b["kernel"]
    for k in ("acc", "theta", "ll", "ra", "nacc", "theta_hist", "prop_hist", "ll_hist"):
        assert np.array_equal(a[k], b[k]), k


def test_chol_rtc_accept_only_and_launch_splits(oracle):
    """The run-time compiled kernel (D = 20) with accept-only histories, a ragged chain
    count and launches of 1, 7 and 64 steps: the same bits as one full-history launch."""
    w = _corr(20, 17)
    o = run_oracle(oracle, w, 999, 50)
    for spl in (1, 7, 64):
        e = run_engine(w, 999, 50, hist=L.HIST_ACCEPT_ONLY, spl=spl)
        assert "[hiprtc]" in e["kernel"] and "ACCEPT_ONLY" in e["kernel"]
        assert_bitwise(e, o, full=False)


@pytest.mark.parametrize("D", [27, 33, 49])
def test_chol_rtc_at_odd_dimensions(oracle, D):
    """Odd D (round 3: one-double scalar-load chunks, above the compile budget, so the
    general kernel ran them) now streams 16-double chunks like any D: the run-time
    chol kernel, bitwise against the oracle; the compile (or cache load) time is
    reported by emcmc_rtc_info and printed."""
    from extensible_mcmc.engine import Engine, EngineConfig

    w = _corr(D, D)
    e = run_engine(w, 640, 30)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},") and "[hiprtc]" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 640, 30))
    eng = Engine(EngineConfig(dim=D, num_chains=64, num_mcmc_steps=2, seed=1))
    eng.add_gaussian_rw_update(np.arange(D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((64, D)))
    origin, secs = eng.rtc_info()
    print(f"D={D}: {eng.kernel_name()} obtained from {origin} in {secs:.2f} s")
    assert origin in ("process", "disk", "compiled")
    eng.close()


_FRESH = r"""
import json, sys, time
sys.path[:0] = [{root!r}, {root!r} + "/extensiblemcmc.jl_amd"]
import numpy as np
from extensible_mcmc.engine import Engine, EngineConfig
D = {D}
rng = np.random.default_rng(148)
A = rng.standard_normal((D, D)); S = A @ A.T / D + np.eye(D)
e = Engine(EngineConfig(dim=D, num_chains=256, num_mcmc_steps=4, seed=1))
t0 = time.perf_counter()  # after the HIP runtime's own start-up
e.add_gaussian_rw_update(np.arange(D), 0.01 * S)
e.set_gsn_target(np.zeros(D), S, rng.standard_normal((10, D)))
e.set_state(np.zeros((256, D)))
dt = time.perf_counter() - t0
print(json.dumps({{"kernel": e.kernel_name(), "rtc": e.rtc_info(), "setup_s": dt}}))
"""


def test_rtc_code_objects_load_from_disk_in_a_fresh_process(tmp_path):
    """The on-disk code-object cache: a run-time chol kernel at D = 48 (a 1–2 minute
    compile) is compiled at most once; a second, fresh process loads it from the
    cache and its handle is ready in under a second (compile time logged)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parents[1])
    env = {"EMCMC_RTC_CACHE": str(tmp_path / "cache")}
    import os
    env = dict(os.environ, **env)
    src = _FRESH.format(root=root, D=48)

    def fresh():
        r = subprocess.run([sys.executable, "-c", src], env=env, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    first = fresh()
    second = fresh()
    print("first", first, "second", second)
    assert first["kernel"].startswith("rwm_gsn_chol_kernel<D=48,") and first["rtc"][0] == "compiled"
    assert second["rtc"][0] == "disk" and second["rtc"][1] < 1.0 and second["setup_s"] < 1.0
    assert any(p.suffix == ".co" for p in (tmp_path / "cache").iterdir())


@pytest.mark.parametrize("D,ll_mode,nobs", [(53, L.LL_PER_OBS, 7), (56, L.LL_SUFFSTAT, 10), (64, L.LL_PER_OBS, 1)])
def test_chol_shared_sweep_shapes(oracle, D, ll_mode, nobs):
    """D ≥ 52 (rwm_gsn_chol_kernel's shared sweep: ltd and every observation through one
    copy of the substitution code) at an odd observation count, the x̄ term and a single
    observation, bitwise against the oracle."""
    w = _corr(D, 7 * D, nobs=nobs)
    e = run_engine(w, 768, 24, ll_mode=ll_mode)
    assert e["kernel"].startswith(f"rwm_gsn_chol_kernel<D={D},") and "[hiprtc]" in e["kernel"]
    assert_bitwise(e, run_oracle(oracle, w, 768, 24, ll_mode=ll_mode))
