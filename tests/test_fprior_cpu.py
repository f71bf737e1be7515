"""The fused diagonal step with a separable prior, host side on CPU (no device):
emcmc_prebuild_fused_prior_kernel compiles rwm_gsn_diag_kernel + FusedPrior (emcmc_fprior.h) for
an update's prior into the on-disk cache — both occupancies select_fused_prior may take — and
refuses the shapes the kernel does not serve (they run on the schedule kernels)."""
import numpy as np
import pytest

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine

N_, G_, U_, MV_, P_ = L.DIST_NORMAL, L.DIST_GAMMA, L.DIST_UNIFORM, L.DIST_MVNORMAL, L.DIST_PRODUCT


@pytest.fixture
def cache(tmp_path, monkeypatch):
    d = tmp_path / "rtc"
    monkeypatch.setenv("EMCMC_RTC_CACHE", str(d))
    return d


@pytest.mark.parametrize("D,lanes", [(32, 0), (16, 0), (24, 0), (32, 1)])
def test_prebuild_compiles_both_occupancies(cache, D, lanes):
    u, keep = Engine.gaussian_rw_desc(range(D), 0.01 * np.eye(D), prior=L.PRIOR_PRODUCT,
                                      prior_factors=[(P_, D, [(N_, 0.0, 2.0), (G_, 3.0, 1.0)] * (D // 2))])
    L.prebuild_fused_prior_kernel(D, u, lanes_per_chain=lanes)
    assert len(list(cache.glob("*.co"))) == 2


def test_standard_prior_of_a_product(cache):
    D = 64
    u, keep = Engine.gaussian_rw_desc(range(D), 0.01 * np.eye(D), prior=L.PRIOR_STANDARD,
                                      prior_factors=[(P_, D, [(N_, 0.0, 2.0)] * D)])
    L.prebuild_fused_prior_kernel(D, u, history_mode=L.HIST_ACCEPT_ONLY, ll_mode=L.LL_SUFFSTAT, unit_target=False)
    assert len(list(cache.glob("*.co"))) == 2


@pytest.mark.parametrize("pos,prior", [([1] * 32, L.PRIOR_IMPROPER), ([j % 4 != 3 for j in range(32)],
                                                                      L.PRIOR_IMPROPER_POS), (None, L.PRIOR_PRODUCT)])
def test_uniform_random_walks(cache, pos, prior):
    D = 32
    fac = [(P_, D, [(G_, 2.0, 1.0)] * D)] if prior == L.PRIOR_PRODUCT else None
    u, keep = Engine.uniform_rw_desc(range(D), [0.05 + 0.001 * j for j in range(D)], pos=pos, prior=prior,
                                     prior_factors=fac)
    L.prebuild_fused_prior_kernel(D, u)
    assert len(list(cache.glob("*.co"))) == 2


@pytest.mark.parametrize("D,lanes,prior", [(32, 0, L.PRIOR_STANDARD), (32, 1, L.PRIOR_PRODUCT), (16, 0, L.PRIOR_STANDARD),
                                           (32, 4, L.PRIOR_STANDARD)])
def test_mvnormal_prior(cache, D, lanes, prior):
    """One MvNormal over all D on one, two or four lanes per chain."""
    u, keep = Engine.gaussian_rw_desc(range(D), 0.01 * np.eye(D), prior=prior,
                                      prior_factors=[(MV_, D, np.zeros(D), np.eye(D) + 0.1 * np.ones((D, D)))])
    L.prebuild_fused_prior_kernel(D, u, lanes_per_chain=lanes)
    assert len(list(cache.glob("*.co"))) == 2


@pytest.mark.parametrize("D,lanes,mvn", [(48, 2, False), (48, 0, True), (24, 2, False)])
def test_refuses_lane_splits_of_the_canonical_sum(cache, D, lanes, mvn):
    """Two lanes of 24 (or 12), three of 16 (auto at D = 48): the likelihood's blocks of 8 under a
    pairwise tree do not split into one subtree per lane (D/LPC must be 8·2^k, LPC ∈ {1, 2, 4})."""
    fac = [(MV_, D, np.zeros(D), np.eye(D))] if mvn else [(P_, D, [(N_, 0.0, 2.0)] * D)]
    u, keep = Engine.gaussian_rw_desc(range(D), 0.01 * np.eye(D), prior=L.PRIOR_STANDARD, prior_factors=fac)
    with pytest.raises(L.EMCMCError) as e:
        L.prebuild_fused_prior_kernel(D, u, lanes_per_chain=lanes)
    assert "not a fused-prior shape" in str(e.value)


@pytest.mark.parametrize("pos,prior", [([1] * 32, L.PRIOR_IMPROPER), ([j % 2 for j in range(32)], L.PRIOR_IMPROPER_POS)])
def test_gaussian_random_walk_with_pos_flags(cache, pos, prior):
    """GaussianRandomWalk's positivity round trips on the fused kernel (ImproperPrior too: the
    flags alone take it off the plain fused kernel)."""
    u, keep = Engine.gaussian_rw_desc(range(32), 0.001 * np.eye(32), pos=pos, prior=prior)
    L.prebuild_fused_prior_kernel(32, u)
    assert len(list(cache.glob("*.co"))) == 2


@pytest.mark.parametrize("case", ["mvnormal_part", "dims1", "asymmetric", "gaussian_asym_pos", "uniform_asym_pos", "adaptive", "dense",
                                  "subset", "improper"])
def test_refuses_other_shapes(cache, case):
    D = 32
    coords, sigma = range(D), 0.01 * np.eye(D)
    pri, fac, pos = L.PRIOR_PRODUCT, [(P_, D, [(N_, 0.0, 2.0)] * D)], None
    if case == "mvnormal_part":  # an MvNormal over 16 of the 32 slots beside a Product
        pri, fac = L.PRIOR_PRODUCT, [(MV_, 16, np.zeros(16), np.eye(16)), (P_, 16, [(N_, 0.0, 2.0)] * 16)]
    elif case == "dims1":  # ProductPrior([Normal]*32, [1]*32): every factor reads θ[1] (priors.jl:64-79)
        fac = [(N_, 1, 0.0, 2.0)] * D
    elif case == "asymmetric":  # a Gamma on lane 0's coordinate 3 only (two lanes of 16)
        comps = [(N_, 0.0, 2.0)] * D
        comps[3] = (G_, 2.0, 1.0)
        fac = [(P_, D, comps)]
    elif case == "gaussian_asym_pos":  # flags on lane 1's coordinates only
        pos = [j >= 16 for j in range(D)]
    elif case == "uniform_asym_pos":  # flags on lane 0's coordinates only
        pos = [j < 16 for j in range(D)]
    elif case == "dense":
        sigma = 0.01 * (np.eye(D) + 0.1 * np.ones((D, D)))
    elif case == "subset":
        coords, sigma = range(8), 0.01 * np.eye(8)
        fac = [(P_, 8, [(N_, 0.0, 2.0)] * 8)]
    elif case == "improper":
        pri, fac = L.PRIOR_IMPROPER, None
    if case == "uniform_asym_pos":
        u, keep = Engine.uniform_rw_desc(coords, 0.1, pos=pos, prior=pri, prior_factors=fac)
    elif case == "adaptive":
        adapt = dict(k=20, target=0.234, scale=0.02, min=1e-12, max=1e7, offset=100.0)
        u, keep = Engine.uniform_rw_desc(coords, 0.1, adapt=adapt, prior=pri, prior_factors=fac)
    else:
        u, keep = Engine.gaussian_rw_desc(coords, sigma, pos=pos, prior=pri, prior_factors=fac)
    with pytest.raises(L.EMCMCError) as e:
        L.prebuild_fused_prior_kernel(D, u)
    assert e.value.status == L.INVALID_ARG
    assert "not a fused-prior shape" in str(e.value)
    assert not list(cache.glob("*.co"))
