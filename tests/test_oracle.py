"""Oracle self-checks (CPU): the shared variate stream and canonical arithmetic.

Pins: Random123 Philox KATs (tests/golden/philox_kat.json); accuracy of the
restated log / exp against numpy; the 8192-strip N(0,1) and 256-strip Exp(1) ziggurat tables (equal strip
areas) and the N(0,1) / Exp(1) distributions they produce; the canonical
Cholesky and summation against LAPACK / math.fsum; and the claim the kernels
rely on that the dense (general-L) formulas give the same bits as the diagonal
ones when Σ is diagonal.
"""
import json
import math

import numpy as np
import pytest

from extensible_mcmc import workloads as W


def test_philox_kat(oracle, golden_dir):
    for v in json.loads((golden_dir / "philox_kat.json").read_text()):
        assert [int(x) for x in oracle.philox(v["ctr"], v["key"])] == v["out"]


def test_log_accuracy(oracle):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(2.0 ** -53, 1.0, 200_000), 2.0 ** -np.arange(0, 54),
                        rng.uniform(0.5, 2.0, 50_000), np.exp(rng.uniform(-700, 700, 50_000)), [1.0]])
    y = oracle.log_vec(x)
    ref = np.log(x)
    nz = ref != 0
    ulp = np.abs(y[nz] - ref[nz]) / np.spacing(np.abs(ref[nz]))
    assert ulp.max() <= 1.0
    assert y[x == 1.0][0] == 0.0


def test_exp_accuracy(oracle):
    rng = np.random.default_rng(3)
    x = np.concatenate([-rng.uniform(0, 8, 200_000), -rng.uniform(0, 700, 50_000), [0.0, -1e-300, -0.5, -700.0]])
    y = oracle.exp_nonpos_vec(x)
    ref = np.exp(x)
    assert (np.abs(y - ref) / ref).max() < 4e-16
    assert y[x == 0.0][0] == 1.0


R_N, V_N = 4.548600609949139, 1.5303723494629906e-4  # 8192-strip normal table (oracle_math.h)


def test_ziggurat_normal_table(oracle):
    """8192 strips of equal area v (M&T construction) as 8-byte edges: an[0] = 0,
    an[j] = x_j increasing to x_{L-1} = r, an[L] = q = v/f(r) (base strip); a
    layer's (bound, width) pair is (an[j-1], an[j]), so every bound is below its
    width (the top strip's bound is 0: it never fast-accepts)."""
    t = oracle.zig_tables()
    an, fn, L = t["an"], t["fn"], 8192
    assert len(an) == L + 2 and an[0] == 0.0 and fn[0] == 1.0
    x = an[1:L]  # x_1 .. x_{L-1}
    assert x[-1] == R_N and np.all(np.diff(x) > 0)
    assert np.allclose(fn[1:L], np.exp(-0.5 * x * x), rtol=1e-14)
    areas = x * (fn[0:L - 1] - fn[1:L])  # strip j spans f(x_j)..f(x_{j-1})
    assert np.allclose(areas, V_N, rtol=1e-9)
    assert an[L] * np.exp(-0.5 * R_N * R_N) == pytest.approx(V_N, rel=1e-12)  # base width q
    assert np.all(an[0:L] < an[1:L + 1])  # bound < width for every layer (base: r < q)


def test_ziggurat_tables(oracle):
    """Strips of equal area v (M&T construction) — 256 for Exp(1), 52-bit
    magnitudes: x_{L-1} = r, top strip reaches x_0 ≈ 0, thresholds below 2^bits
    and increasing towards the base."""
    t = oracle.zig_tables()
    for k, w, f, r, v, fx, L, m in ((t["ke"], t["we"], t["fe"], 7.69711747013104972, 3.949659822581572e-3,
                                     lambda x: np.exp(-x), 256, 2.0 ** 52),):
        assert len(k) == L
        x = w * m  # x_i for i ≥ 1; base strip width for i = 0
        assert x[L - 1] == pytest.approx(r, rel=1e-15)
        assert np.all(np.diff(x[1:]) > 0)
        assert np.allclose(f[1:], fx(x[1:]), rtol=1e-14)
        areas = x[1:] * (f[:-1] - f[1:])  # strip i spans f(x_i)..f(x_{i-1})
        assert np.allclose(areas, v, rtol=1e-9)
        assert x[0] * fx(r) == pytest.approx(v, rel=1e-12)  # base rectangle width q
        assert k[1] == 0 and np.all(k < m)
        assert np.allclose(k[2:] / m, x[1:-1] / x[2:], rtol=1e-15, atol=1.0 / m)


def test_ziggurat_normal_constants_close_the_table():
    """r, v of the 8192-strip normal table: v = r·f(r) + ∫_r^∞ f, and the
    recursion from x = r up through the strips ends with the top strip's area
    equal to v (checked in 50-digit arithmetic)."""
    import mpmath as mp

    mp.mp.dps = 50
    r, v = mp.mpf(R_N), mp.mpf(V_N)
    f = lambda x: mp.e ** (-x * x / 2)  # noqa: E731
    assert abs(r * f(r) + mp.sqrt(2 * mp.pi) * mp.ncdf(-r) - v) / v < 1e-14  # r, v rounded to double
    x = r
    for _ in range(8192 - 2):
        x = mp.sqrt(-2 * mp.log(v / x + f(x)))
    assert abs(x * (1 - f(x)) - v) / v < 1e-9


def test_ziggurat_distributions(oracle):
    from scipy import stats

    z = oracle.normals(W.SEED, 400_000)
    assert abs(z.mean()) < 0.006 and abs(z.std() - 1.0) < 0.006
    assert stats.kstest(z, "norm").pvalue > 1e-3
    # tail beyond r = 4.55 is reached through the rare path and has the right mass
    tail = (np.abs(z) > R_N).mean()
    assert abs(tail - 2 * stats.norm.sf(R_N)) < 2e-5
    assert tail > 0
    e = oracle.exponentials(W.SEED, 200_000)
    assert abs(e.mean() - 1.0) < 0.01
    assert stats.kstest(e, "expon").pvalue > 1e-3
    assert (e > 7.69711747013104972).sum() > 0


def test_variates_depend_on_counter(oracle):
    a = oracle.step_variates(W.SEED, 3, 7, 4)
    b = oracle.step_variates(W.SEED, 3, 7, 4)
    c = oracle.step_variates(W.SEED, 4, 7, 4)
    d = oracle.step_variates(W.SEED + 1, 3, 7, 4)
    e = oracle.step_variates(W.SEED, 3, 7, 4, pidx0=1)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]
    for other in (c, d, e):
        assert not np.array_equal(a[0], other[0])


def test_cholesky_matches_lapack(oracle):
    rng = np.random.default_rng(2)
    for D in (1, 2, 5, 32):
        A = rng.standard_normal((D, D))
        S = A @ A.T + D * np.eye(D)
        L = oracle.cholesky(S)
        assert np.allclose(L, np.linalg.cholesky(S), rtol=1e-13, atol=1e-13)
        # only the upper triangle is read (Symmetric(Σ), uplo = :U)
        S2 = np.triu(S) + np.tril(rng.standard_normal((D, D)), -1)
        assert np.array_equal(oracle.cholesky(S2), L)
    with pytest.raises(np.linalg.LinAlgError):
        oracle.cholesky(np.array([[1.0, 2.0], [2.0, 1.0]]))


@pytest.mark.parametrize("D", [1, 2, 3, 8, 16, 24, 32, 64])
def test_canonical_sum(oracle, D):
    rng = np.random.default_rng(D)
    v = rng.uniform(0, 1, D)
    s = oracle.canon_sum(v)
    assert abs(s - math.fsum(v)) <= 4 * D * np.spacing(s)
    blk = 8 if (D % 8 == 0 and D >= 16) else D
    parts = [sum_seq(v[i:i + blk]) for i in range(0, D, blk)]
    while len(parts) > 1:
        nxt = [parts[2 * i] + parts[2 * i + 1] for i in range(len(parts) // 2)]
        if len(parts) % 2:
            nxt.append(parts[-1])
        parts = nxt
    assert s == parts[0]


def sum_seq(v):
    s = v[0]
    for x in v[1:]:
        s = s + x
    return s


@pytest.mark.parametrize("ll_mode", [0, 1])
def test_dense_formulas_equal_diagonal_bits(oracle, ll_mode):
    w = W.cfg2(16)
    runs = []
    for force_dense in (0, 0x100):
        st = oracle.OracleState(np.zeros((16, w.D)))
        h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1,
                           nsteps=60, ll_mode=ll_mode | force_dense)
        runs.append((st, h))
    (a, ha), (b, hb) = runs
    assert np.array_equal(ha["acc"], hb["acc"])
    assert np.array_equal(ha["ll"], hb["ll"])
    assert np.array_equal(ha["theta"], hb["theta"])
    assert np.array_equal(a.ra, b.ra)


def test_markstein_quotient_is_ieee_division(oracle):
    """The kernels divide the rolling-acceptance numerator by W (N ≥ W) with
    Markstein's correction from RN(1/W); it must round like IEEE division."""
    rng = np.random.default_rng(11)
    n = 400_000
    x = np.ldexp(1.0 + rng.integers(0, 2 ** 52, n) * 2.0 ** -52, rng.integers(-60, 200, n))
    x[rng.random(n) < 0.5] *= -1
    ints = rng.integers(-1_000_000, 1_000_001, n // 4).astype(np.float64)
    halves = rng.integers(-256, 257, n // 4) / 2.0
    xs = np.concatenate([x, ints, halves])
    for b in list(range(1, 129)):
        assert oracle.markstein_mismatches(b, xs if b in (1, 7, 100, 127, 128) else xs[::16]) == 0


def _ulps(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    return np.abs(ia - ib)


def test_exp_le0_table_driven(oracle):
    """The MALA exp: ≤ 1 ulp against 50-digit e^x on random x ≤ 0 (normal
    results), IEEE-rounded subnormals, 0 below −745.13, NaN kept."""
    import mpmath as mp

    rng = np.random.default_rng(5)
    x = np.concatenate([-rng.exponential(3.0, 4000), -rng.uniform(0, 700, 2000), [0.0, -0.0, -1e-300, -np.log(2)]])
    y = oracle.exp_le0_vec(x)
    mp.mp.dps = 40
    ref = np.array([float(mp.e ** mp.mpf(v)) for v in x])
    assert _ulps(y, ref).max() <= 1
    sub = np.array([-709.0, -720.0, -740.0, -745.0, -745.2, -800.0, -np.inf])
    ys = oracle.exp_le0_vec(sub)
    refs = np.array([float(mp.e ** mp.mpf(v)) if np.isfinite(v) else 0.0 for v in sub])
    assert np.all(np.abs(ys - refs) <= 2 * 5e-324 + 2.3e-16 * refs)
    assert np.isnan(oracle.exp_le0_vec(np.array([np.nan]))[0])


def test_log_1_2_table_driven(oracle):
    """The MALA log on [1, 2]: relative error ≤ 1.5 ulp away from 1, absolute
    error ≤ 2^-60 near 1 (the log-likelihood adds it to O(1) terms)."""
    import mpmath as mp

    rng = np.random.default_rng(6)
    u = np.concatenate([1.0 + rng.random(6000), 1.0 + np.exp(-rng.uniform(0, 40, 2000)), [1.0, 2.0, 1.5, np.nextafter(2.0, 0)]])
    y = oracle.log_1_2_vec(u)
    mp.mp.dps = 40
    ref = np.array([float(mp.log(mp.mpf(v))) for v in u])
    err = np.abs(y - ref)
    far = u > 1.01
    assert np.all(err[far] <= 1.5 * np.spacing(ref[far]))
    assert np.all(err <= 2.0 ** -60 + 1.5 * np.spacing(ref))
    assert oracle.log_1_2_vec(np.array([1.0]))[0] == 0.0 or abs(oracle.log_1_2_vec(np.array([1.0]))[0]) < 2 ** -60


def test_rcp_1_2_table_driven(oracle):
    """The MALA logistic terms' 1/u on [1, 2] (no division: the log reduction's
    RN(1/c_j) times a degree-6 series in r): within 2 ulp of the exact quotient,
    exact at u = 1 and u = 2."""
    rng = np.random.default_rng(7)
    u = np.concatenate([1.0 + rng.random(20000), 1.0 + np.exp(-rng.uniform(0, 40, 4000)),
                        1.0 + np.arange(129) / 128.0, [np.nextafter(2.0, 0), np.nextafter(1.0, 2)]])
    y = oracle.rcp_1_2_vec(u)
    ref = 1.0 / u  # IEEE division: correctly rounded, within 0.5 ulp of the true quotient
    assert np.all(np.abs(y - ref) <= 2.0 * np.spacing(ref))
    assert oracle.rcp_1_2_vec(np.array([1.0, 2.0])).tolist() == [1.0, 0.5]


def test_faithful_refactor_variant_has_the_same_bits(oracle):
    """The CPU baseline's "faithful" variant (a Cholesky per MvNormal construction,
    random_walk.jl:147,167, gsn_target.jl:20) gives the factor-once path's bits."""
    from extensible_mcmc import workloads as W

    w = W.cfg2(64, D=32)
    runs = []
    for mode in (0, 0x200):
        st = oracle.OracleState(np.zeros((64, w.D)))
        h = oracle.run_gsn(st, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=60,
                           ll_mode=mode)
        runs.append((st, h))
    (a, ha), (b, hb) = runs
    assert np.array_equal(a.theta, b.theta) and np.array_equal(a.ll, b.ll) and np.array_equal(a.ra, b.ra)
    for k in ("theta", "prop", "ll", "acc"):
        assert np.array_equal(ha[k], hb[k]), k


def test_accept_only_mode_matches_full_history(oracle):
    """run_gsn / run_mix accept_only=True: the same accept stream and final state as a
    full-history call (the θ/θ°/ll buffers are optional outputs of the same loop), and
    pack_accept / accept_mismatch_chains agree with the unpacked comparison."""
    from extensible_mcmc import workloads as W

    w = W.cfg2(200)
    a = oracle.OracleState(np.zeros((200, 32)))
    b = oracle.OracleState(np.zeros((200, 32)))
    ha = oracle.run_gsn(a, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=30)
    hb = oracle.run_gsn(b, seed=w.seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=30,
                        accept_only=True)
    assert set(hb) == {"acc"} and np.array_equal(ha["acc"], hb["acc"])
    assert np.array_equal(a.theta, b.theta) and np.array_equal(a.ll, b.ll) and np.array_equal(a.ra, b.ra)
    pa = oracle.pack_accept(ha["acc"])
    assert pa.shape == (30, 4) and pa.dtype == np.uint64
    assert oracle.accept_mismatch_chains(pa, oracle.pack_accept(hb["acc"]), 200).size == 0
    flipped = ha["acc"].copy()
    flipped[3, 77] ^= True
    flipped[29, 199] ^= True
    assert list(oracle.accept_mismatch_chains(oracle.pack_accept(flipped), pa, 200)) == [77, 199]
    w4 = W.cfg4(64, k=10)
    m1 = oracle.MixState(np.zeros((64, 32)), sigma_b=w4.sigma_b)
    m2 = oracle.MixState(np.zeros((64, 32)), sigma_b=w4.sigma_b)
    kw = dict(seed=w4.seed, sigma_a=w4.rw_sigma, t_sigma=w4.t_sigma, obs=w4.obs, iter0=1, nsteps=25, lam=w4.lam,
              haario_k=10)
    h1 = oracle.run_mix(m1, **kw)
    h2 = oracle.run_mix(m2, accept_only=True, **kw)
    assert set(h2) == {"acc"} and np.array_equal(h1["acc"], h2["acc"])
    assert np.array_equal(m1.LB, m2.LB) and np.array_equal(m1.cov, m2.cov) and m1.M == m2.M == 25 % 10
