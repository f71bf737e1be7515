"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle on the
same seeds and chain ids.  Bar: bit-exact accept/reject stream, θ, θ°, ll,
rolling acceptance and accept counts (integer and fp64 alike — both sides use
the same IEEE operation sequence)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc import workloads as W
from extensible_mcmc.engine import Engine, EngineConfig

from helpers import assert_bitwise, run_engine, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def test_device_log_matches_oracle(oracle):
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(2.0 ** -53, 1.0, 500_000), 2.0 ** -np.arange(0, 54),
                        np.exp(rng.uniform(-700, 700, 100_000)), [1.0, 0.5, 2.0]])
    assert np.array_equal(L.probe_log(x), oracle.log_vec(x))


@pytest.mark.parametrize("D", [1, 2, 3, 32])
def test_device_variates_match_oracle(oracle, D):
    rng = np.random.default_rng(D)
    n = 4096
    chains = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    iters = rng.integers(1, 2 ** 31, n, dtype=np.uint64).astype(np.uint32)
    z, E = L.probe_variates(W.SEED, chains, iters, D)
    for i in range(0, n, 7):
        zo, Eo, _ = oracle.step_variates(W.SEED, int(chains[i]), int(iters[i]), D)
        assert np.array_equal(z[i], zo)
        assert E[i] == Eo


def test_device_variates_cover_every_ziggurat_path(oracle):
    """2M normals and 32k accept exponentials of one chain, all bitwise equal to the
    oracle, including the rare paths: N(0,1) draws beyond the base strip's edge r
    (tail, ≈ 5e-6 per draw), draws from wedges (≈ 6e-4) and Exp(1) draws past
    its r."""
    R_N, R_E = 4.548600609949139, 7.69711747013104972
    n, D, chain, it0 = 32768, 64, 12345, 1000
    z, E = L.probe_variates(W.SEED, np.full(n, chain, np.uint32), np.arange(it0, it0 + n, dtype=np.uint32), D)
    zo = oracle.normals(W.SEED, n * D, chain=chain, iter0=it0).reshape(n, D)
    assert np.array_equal(z, zo)
    assert (np.abs(z) > R_N).sum() >= 2  # tail path taken (expected ≈ 11)
    Eo = np.array([oracle.step_variates(W.SEED, chain, int(i), 1)[1] for i in range(it0, it0 + 2048)])
    assert np.array_equal(E[:2048], Eo)
    En = L.probe_variates(W.SEED, np.arange(1, 2 ** 20 + 1, dtype=np.uint32), np.full(2 ** 20, 7, np.uint32), 1)[1]
    assert np.array_equal(En, oracle.exponentials(W.SEED, 2 ** 20, chain0=1, it=7))
    assert (En > R_E).sum() > 0 and abs(En.mean() - 1.0) < 0.005  # Exp(1) tail path taken


@pytest.mark.parametrize("lpc", [1, 2, 4])
@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
def test_d32_headline_shape(oracle, lpc, ll_mode):
    w = W.cfg2(2048)
    e = run_engine(w, 2048, 150, lpc=lpc, ll_mode=ll_mode)
    assert f"LPC={lpc}" in e["kernel"]
    o = run_oracle(oracle, w, 2048, 150, ll_mode=ll_mode)
    assert_bitwise(e, o)


def test_d32_accept_only_and_launch_splits(oracle):
    w = W.cfg2(1000)  # 1000 chains: partial last wave at every LPC
    o = run_oracle(oracle, w, 1000, 130)
    for spl in (1, 7, 64):
        e = run_engine(w, 1000, 130, lpc=4, hist=L.HIST_ACCEPT_ONLY, spl=spl)
        assert "ACCEPT_ONLY" in e["kernel"]
        assert_bitwise(e, o, full=False)


@pytest.mark.parametrize("which", ["ref_test", "iso"])
def test_d2_reference_test_target(oracle, which):
    w = W.ref_test() if which == "ref_test" else W.cfg1(True)
    e = run_engine(w, 777, 300)
    assert ("dense" in e["kernel"]) == (which == "ref_test")
    o = run_oracle(oracle, w, 777, 300)
    assert_bitwise(e, o)


@pytest.mark.parametrize("D,lpc", [(16, 2), (64, 4), (8, 1), (3, 1)])
def test_other_dims(oracle, D, lpc):
    w = W.cfg2(512, D=D)
    e = run_engine(w, 512, 80, lpc=lpc)
    o = run_oracle(oracle, w, 512, 80)
    assert_bitwise(e, o)


def test_dense_correlated_d4(oracle):
    rng = np.random.default_rng(4)
    A = rng.standard_normal((4, 4))
    S = A @ A.T / 4 + np.eye(4)
    B = rng.standard_normal((4, 4))
    R = 0.1 * (B @ B.T / 4 + np.eye(4))
    obs = rng.multivariate_normal(np.ones(4), S, size=9)
    w = W.GsnWorkload("d4", 4, 300, np.ones(4), S, R, obs, np.zeros(4))
    for ll_mode in (0, 1):
        e = run_engine(w, 300, 120, ll_mode=ll_mode)
        assert "dense" in e["kernel"]
        assert_bitwise(e, run_oracle(oracle, w, 300, 120, ll_mode=ll_mode))


def test_shard_offsets_reproduce_unsharded_chains(oracle):
    """Chains keyed by global id: two shards == one run (the 8-GPU invariant)."""
    w = W.cfg5(4096)
    full = run_engine(w, 4096, 60, theta0=w.theta_init[:4096])
    a = run_engine(w, 2048, 60, chain0=0, theta0=w.theta_init[:2048])
    b = run_engine(w, 2048, 60, chain0=2048, theta0=w.theta_init[2048:4096])
    assert np.array_equal(np.concatenate([a["theta"], b["theta"]]), full["theta"])
    assert np.array_equal(np.concatenate([a["acc"], b["acc"]], axis=1), full["acc"])
    o = run_oracle(oracle, w, 256, 60, chain0=2048, theta0=w.theta_init[2048:2304])
    assert np.array_equal(b["theta"][:256], o["state"].theta)


def test_resume_across_runs(oracle):
    w = W.cfg2(640)
    e = run_engine(w, 640, 50, M=120, fetch=False)
    eng = e["engine"]
    eng.run_iters(51, 70)
    eng.synchronize()
    th, ll = eng.get_state()
    o = run_oracle(oracle, w, 640, 120, history=False)
    assert np.array_equal(th, o["state"].theta)
    assert np.array_equal(ll, o["state"].ll)


def test_nonfinite_target_sets_fault_bit():
    w = W.cfg2(64, D=2)
    w.obs = np.full_like(w.obs, 1e300)  # (x − μ)² overflows → ll° = −Inf
    e = run_engine(w, 64, 5, fetch=False)
    assert (e["faults"] & L.FAULT_NONFINITE_LL).all()
    assert not e["engine"].synchronize(allow_faults=True)


def test_fused_schedule_gap_restarts_rolling_rate(oracle):
    """A schedule gap (iterations 41:60 skipped) on the fused single-update
    kernel: rolling_ar[iter−1] of a skipped iteration reads 0.0
    (chain_statistics.jl:57), in the engine and in the oracle."""
    w = W.cfg2(500)
    eng = Engine(EngineConfig(dim=w.D, num_chains=500, num_mcmc_steps=120, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((500, w.D)))
    eng.run_iters(1, 40)
    eng.run_iters(61, 60)
    eng.synchronize()
    st = oracle.OracleState(np.zeros((500, w.D)))
    iters = np.concatenate([np.arange(1, 41), np.arange(61, 121)]).astype(np.uint32)
    oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=100,
                   iters=iters, nthreads=8, history=False)
    th, ll = eng.get_state()
    ra, _ = eng.get_chain_stats()
    assert np.array_equal(th, st.theta) and np.array_equal(ll, st.ll)
    assert np.array_equal(ra[0], st.ra)


def test_reused_step_array_is_read_at_every_run(oracle):
    """Engine.run keeps the address of a step array it has seen (the driver's repeated
    window): the same array object, refilled in place with the next iterations, and
    then a reshaped one, must run the iterations it holds at each call."""
    w = W.cfg2(320)
    eng = Engine(EngineConfig(dim=w.D, num_chains=320, num_mcmc_steps=100, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((320, w.D)))
    steps = np.ones((20, 2), dtype=np.uint32)
    for k in range(3):  # iterations 1..60 through one array
        steps[:, 0] = np.arange(1 + 20 * k, 21 + 20 * k, dtype=np.uint32)
        eng.run(steps)
    steps[:, 0] = np.arange(61, 81, dtype=np.uint32)
    steps.shape = (10, 4)  # the same object and buffer under another shape: the general path
    eng.run(steps)
    eng.run(np.stack([np.arange(81, 101, dtype=np.uint32), np.ones(20, np.uint32)], axis=1))
    eng.synchronize()
    st = oracle.OracleState(np.zeros((320, w.D)))
    oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=100,
                   nthreads=8, history=False)
    th, ll = eng.get_state()
    assert np.array_equal(th, st.theta) and np.array_equal(ll, st.ll)
    eng.close()


@pytest.mark.parametrize("C", [1, 63, 65, 257])
def test_ragged_and_tiny_chain_counts(oracle, C):
    """One chain, and counts that leave partial waves / blocks at LPC = 2:
    every chain still matches the oracle bit for bit."""
    w = W.cfg2(C)
    e = run_engine(w, C, 40, lpc=2)
    o = run_oracle(oracle, w, C, 40)
    assert_bitwise(e, o)


def test_empty_schedule_is_a_no_op(oracle):
    """emcmc_run with zero steps launches nothing and leaves the state as set."""
    w = W.cfg2(128)
    eng = Engine(EngineConfig(dim=w.D, num_chains=128, num_mcmc_steps=10, seed=w.seed))
    eng.add_gaussian_rw_update(np.arange(w.D), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    th0 = np.random.default_rng(3).standard_normal((128, w.D))
    eng.set_state(th0)
    eng.run(np.zeros((0, 2), dtype=np.uint32))
    eng.synchronize()
    th, ll = eng.get_state()
    assert np.array_equal(th, th0)
    assert np.all(ll == -np.inf)
    eng.close()


@pytest.mark.parametrize("ll_mode", [L.LL_PER_OBS, L.LL_SUFFSTAT])
@pytest.mark.parametrize("unit", [True, False])
def test_scalar_obs_variant_bitwise(oracle, ll_mode, unit):
    """EMCMC_VARIANT_SCALAR_OBS (rwm_gsn_diag_s_kernel: one lane per chain, the
    observation rows as SGPR operands streamed through the scalar cache): the
    same bits as the oracle, with a unit and a non-unit diagonal target Σ,
    1000 chains (a partial last wave) and launch splits."""
    w = W.cfg2(1000)
    if not unit:
        w.t_sigma = np.diag(np.random.default_rng(9).uniform(0.5, 2.0, 32))
    o = run_oracle(oracle, w, 1000, 110, ll_mode=ll_mode)
    for spl in (0, 37):
        e = run_engine(w, 1000, 110, ll_mode=ll_mode, spl=spl, variant=L.VARIANT_SCALAR_OBS)
        assert e["kernel"].startswith("rwm_gsn_diag_s_kernel<D=32,LPC=1")
        assert_bitwise(e, o)


@pytest.mark.parametrize("D,lpc", [(32, 2), (16, 1), (64, 4)])
@pytest.mark.parametrize("variant", [0, L.VARIANT_UNCAPPED])
def test_register_cap_variants_bitwise(oracle, D, lpc, variant):
    """The diag kernel at D = 16 / 32 / 64 is built twice: capped at 256 registers
    (MINW = 2, 512-thread blocks whose sibling waves pace each other — the default)
    and uncapped (EMCMC_VARIANT_UNCAPPED, one wave per SIMD).  Same bits as the
    oracle either way, with 1000 chains (a partial last block) and launch splits."""
    w = W.cfg2(1000, D=D)
    o = run_oracle(oracle, w, 1000, 60)
    for spl in (0, 23):
        e = run_engine(w, 1000, 60, lpc=lpc, spl=spl, variant=variant)
        assert ("MINW=2" in e["kernel"]) == (variant == 0), e["kernel"]
        assert_bitwise(e, o)


def test_many_observations_beyond_lds(oracle):
    """Per-observation likelihood with more observations than the LDS holds
    (600 × 32 doubles = 150 KiB next to the 70 KiB ziggurat): the fused path
    streams them through the scalar cache (rwm_gsn_diag_s_kernel) instead of
    refusing; bitwise against the oracle."""
    w = W.cfg2(512, nobs=600)
    e = run_engine(w, 512, 40)
    assert e["kernel"].startswith("rwm_gsn_diag_s_kernel<D=32")
    assert_bitwise(e, run_oracle(oracle, w, 512, 40))


def test_many_observations_other_dims_use_the_general_kernel(oracle):
    """The same at D = 4 with 6,000 observations (no scalar-cache instantiation):
    the general kernel reads them from global memory; bitwise against its oracle."""
    from test_gpu_mwg import check, full_steps, run_both

    rng = np.random.default_rng(41)
    mu = np.array([0.5, -1.0, 2.0, 0.0])
    obs = mu + rng.standard_normal((6000, 4))
    ups = [oracle.mwg_update(2, [0, 1, 2, 3], sigma=np.eye(4) * 2e-4)]
    steps = full_steps(60, 1)
    eng, st, h = run_both(oracle, 4, 300, 60, ups, mu, np.eye(4), obs, steps, 99)
    assert "mwg_gsn_kernel<D=4" in eng.kernel_name()
    check(oracle, eng, st, h, steps, ups, 1)


def test_state_left_in_history_feeds_the_next_kernel():
    """After a FULL-history run of the fused diagonal kernel the current θ lives in its
    last history slot (emcmc.hip theta_live; the state buffer is not written back): a
    later run on another kernel — a dense Σ_t selects rwm_gsn_chol_kernel — and
    get_state must both see it.  The same second part started from get_state's θ on a
    fresh engine gives the same chains, bit for bit."""
    rng = np.random.default_rng(41)
    w = W.cfg2(512, D=16)
    A = rng.standard_normal((16, 16))
    St = A @ A.T / 16 + np.eye(16)
    eng = Engine(EngineConfig(dim=16, num_chains=512, num_mcmc_steps=60, seed=w.seed, steps_per_launch=7))
    eng.add_gaussian_rw_update(np.arange(16), w.rw_sigma)
    eng.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    eng.set_state(np.zeros((512, 16)))
    eng.run_iters(1, 30)
    eng.synchronize()
    assert eng.kernel_name().startswith("rwm_gsn_diag_kernel")
    th_mid, ll_mid = eng.get_state()
    last = eng.get_history(L.H_STATE, 30, 1)[0, 0]
    assert np.array_equal(th_mid, last)  # the state is the last history slot
    eng.run_iters(31, 5)  # fused again: starts from the slot, leaves θ in slot 35
    eng.set_gsn_target(w.mu_true, St, w.obs)
    eng.run_iters(36, 20)
    eng.synchronize()
    assert "chol" in eng.kernel_name()
    th_a, _ = eng.get_state()

    ref = Engine(EngineConfig(dim=16, num_chains=512, num_mcmc_steps=60, seed=w.seed, steps_per_launch=7))
    ref.add_gaussian_rw_update(np.arange(16), w.rw_sigma)
    ref.set_gsn_target(w.mu_true, w.t_sigma, w.obs)
    ref.set_state(th_mid, ll_mid)
    ref.run_iters(31, 5)
    ref.synchronize()
    th5, ll5 = ref.get_state()
    ref.set_gsn_target(w.mu_true, St, w.obs)
    ref.set_state(th5, ll5)
    ref.run_iters(36, 20)
    ref.synchronize()
    th_b, _ = ref.get_state()
    assert np.array_equal(th_a, th_b)
