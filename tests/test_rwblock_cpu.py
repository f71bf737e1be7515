"""mwg_rw_block_kernel's host side on CPU (no device): emcmc_prebuild_rw_block_kernel
compiles the kernel for an update's structure (emcmc.hip rw_shape_source → hiprtc)
into an on-disk cache, and refuses a shape the kernel does not serve."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine


@pytest.fixture
def cache(tmp_path, monkeypatch):
    d = tmp_path / "rtc"
    monkeypatch.setenv("EMCMC_RTC_CACHE", str(d))
    return d


def test_prebuild_compiles_a_shape_into_the_cache(cache):
    D = 17
    u, keep = Engine.uniform_rw_desc(range(D), 0.1, pos=[j % 2 for j in range(D)], prior=L.PRIOR_PRODUCT,
                                     prior_factors=[(L.DIST_PRODUCT, D, [(L.DIST_GAMMA, 2.0, 1.0)] * D)])
    L.prebuild_rw_block_kernel(D, u, history_mode=L.HIST_ACCEPT_ONLY)
    assert len(list(cache.glob("*.co"))) == 1


def test_prebuild_compiles_a_two_update_schedule(cache):
    """Metropolis-within-Gibbs: two GaussianRandomWalk blocks over interleaved coordinates, one
    with a ProductPrior, one reversed — one kernel for the schedule."""
    D = 24
    a, ka = Engine.gaussian_rw_desc(range(0, D, 2), 0.01 * np.eye(D // 2), prior=L.PRIOR_PRODUCT,
                                    prior_factors=[(L.DIST_PRODUCT, D // 2, [(L.DIST_NORMAL, 0.0, 1.0)] * (D // 2))])
    b, kb = Engine.gaussian_rw_desc(list(range(1, D, 2))[::-1], 0.01 * np.eye(D // 2))
    L.prebuild_rw_block_kernel(D, [a, b])
    assert len(list(cache.glob("*.co"))) == 1


@pytest.mark.parametrize("case", ["mix", "small_d", "mala", "gaussian_pos_64", "gaussian_pos_33"])
def test_prebuild_refuses_other_shapes(cache, case):
    """... and a GaussianRandomWalk with more than 32 positivity flags: its round trips always need
    scratch, and at 64 flags the gfx950 backend aborts the compiling process — the shape is refused
    before hiprtc sees it (the wide kernel runs it)."""
    D = {"small_d": 8, "gaussian_pos_64": 64, "gaussian_pos_33": 40}.get(case, 20)
    coords = range(D)
    if case.startswith("gaussian_pos"):
        n = 64 if case == "gaussian_pos_64" else 33
        u, keep = Engine.gaussian_rw_desc(range(n), 0.001 * np.eye(n), pos=[1] * n)
    elif case == "mala":
        u = L.EmcmcUpdateDesc()
        u.kernel = L.MALA
        c = np.arange(D, dtype=np.uint32)
        e = np.array([0.1])
        u.num_coords, u.coords, u.epsilon = D, L.u32ptr(c), L.dptr(e)
        keep = [c, e]
    elif case == "mix":
        u = L.EmcmcUpdateDesc()
        u.kernel = L.RW_GAUSSIAN_MIX
        c = np.arange(D, dtype=np.uint32)
        S = np.ascontiguousarray(np.eye(D).ravel())
        u.num_coords, u.coords, u.sigma, u.sigma_b, u.mix_lambda = D, L.u32ptr(c), L.dptr(S), L.dptr(S), 0.5
        keep = [c, S]
    else:
        u, keep = Engine.gaussian_rw_desc(coords, 0.01 * np.eye(D), prior=L.PRIOR_IMPROPER_POS)
    with pytest.raises(L.EMCMCError) as e:
        L.prebuild_rw_block_kernel(D, u)
    assert e.value.status == L.INVALID_ARG
    assert not list(cache.glob("*.co"))


def test_prebuild_compiles_32_gaussian_pos_flags(cache):
    """The limit's edge: 32 flagged coordinates (every other one of 64) still compile."""
    D = 64
    u, keep = Engine.gaussian_rw_desc(range(D), 0.001 * np.eye(D), pos=[j % 2 for j in range(D)])
    L.prebuild_rw_block_kernel(D, u)
    assert len(list(cache.glob("*.co"))) == 1
