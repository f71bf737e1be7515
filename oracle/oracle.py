"""ctypes wrapper of oracle/lib/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  See oracle/emcmc_oracle.c for what is restated and the parity
status ("parity unpinned" against the Julia reference itself; pinned by the
Random123 KATs, the reference's own schedule/adaptation KATs, the numpy
literal restatement in oracle/literal.py and the analytic posterior).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
import os  # noqa: E402

# EMCMC_ORACLE_LIB: an alternative build (tests/test_oracle_sanitized.py loads the ASan/UBSan one)
LIB_PATH = Path(os.environ.get("EMCMC_ORACLE_LIB", ORACLE_DIR / "lib" / "liboracle.so"))

_lib = None


def build(force: bool = False) -> Path:
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        dp = C.POINTER(C.c_double)
        u32p = C.POINTER(C.c_uint32)
        u64p = C.POINTER(C.c_uint64)
        u8p = C.POINTER(C.c_uint8)
        L.orc_run_gsn.restype = C.c_int
        L.orc_run_gsn.argtypes = [
            C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, dp, dp, C.c_uint64, dp, C.c_int, C.c_uint32,
            u32p, C.c_uint32, C.c_uint32, C.c_uint64, dp, dp, dp, u64p, u32p, u32p, dp, dp, dp, u8p, C.c_int,
        ]
        L.orc_cholesky.restype = C.c_int
        L.orc_cholesky.argtypes = [dp, C.c_int, dp]
        L.orc_canon_sum.restype = C.c_double
        L.orc_canon_sum.argtypes = [dp, C.c_int]
        L.orc_gsn_constants.restype = C.c_int
        L.orc_gsn_constants.argtypes = [C.c_int, dp, dp, C.c_uint64, dp, dp, dp, dp]
        L.orc_philox.restype = None
        L.orc_philox.argtypes = [u32p, u32p, u32p]
        L.orc_step_variates.restype = C.c_uint32
        L.orc_step_variates.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, dp, dp]
        L.orc_log_vec.restype = None
        L.orc_log_vec.argtypes = [dp, dp, C.c_uint64]
        L.orc_exp_nonpos_vec.restype = None
        L.orc_exp_nonpos_vec.argtypes = [dp, dp, C.c_uint64]
        L.orc_normal_vec.restype = None
        L.orc_normal_vec.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, dp]
        L.orc_exp_vec.restype = None
        L.orc_exp_vec.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, dp]
        for nm in ("orc_exp_any_vec", "orc_log_any_vec", "orc_exp_le0_vec", "orc_log_1_2_vec",
                   "orc_rcp_1_2_vec"):
            getattr(L, nm).restype = None
            getattr(L, nm).argtypes = [dp, dp, C.c_uint64]
        L.orc_markstein_mismatches.restype = C.c_uint64
        L.orc_markstein_mismatches.argtypes = [C.c_double, dp, C.c_uint64]
        L.orc_zig_tables_copy.restype = None
        L.orc_zig_tables_copy.argtypes = [dp, dp, u64p, dp, dp]
        _lib = L
    return _lib


def _d(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _colmajor(S, D):
    return np.ascontiguousarray(np.asarray(S, dtype=np.float64).reshape(D, D).ravel(order="F"))


class OracleState:
    """Carried per-chain state (mirrors the engine's SoA state)."""

    def __init__(self, theta, ll=None):
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        self.C, self.D = theta.shape
        self.theta = theta.copy()
        self.ll = np.full(self.C, -np.inf) if ll is None else np.ascontiguousarray(ll, dtype=np.float64).copy()
        self.ra = np.zeros(self.C)
        self.ring = np.zeros((self.C, 2), dtype=np.uint64)
        self.nacc = np.zeros(self.C, dtype=np.uint32)
        self.faults = np.zeros(self.C, dtype=np.uint32)
        self.N = 1  # GenericChainStats.N
        self.last_iter = 0  # last iteration run (rolling_ar[iter−1] reads 0.0 after a gap)


def alloc_history(C, D, nsteps, accept_only=False):
    """History buffers of one oracle call: θ, θ°, ll [nsteps][C](D) and the accept bytes;
    accept_only: the accept bytes alone (1 B per chain-step, so every chain of a
    BASELINE shape replays in memory — the θ/θ°/ll histories are never formed)."""
    if accept_only:
        return {"acc": np.empty((nsteps, C), dtype=np.uint8)}
    return {"theta": np.empty((nsteps, C, D)), "prop": np.empty((nsteps, C, D)), "ll": np.empty((nsteps, C)),
            "acc": np.empty((nsteps, C), dtype=np.uint8)}


def pack_accept(acc):
    """[n][C] accept flags → [n][⌈C/64⌉] u64 words, bit c%64 of word c//64 = chain c: the
    layout of the engine's accept history rows (Engine.get_history_bits)."""
    acc = np.asarray(acc)
    n, C = acc.shape
    words = (C + 63) // 64
    b = np.zeros((n, words * 8), dtype=np.uint8)
    b[:, :(C + 7) // 8] = np.packbits(acc.view(np.uint8) if acc.dtype == bool else acc.astype(np.uint8), axis=1,
                                      bitorder="little")
    return b.view(np.uint64)


def accept_mismatch_chains(got_words, want_words, C):
    """Chains (of C) whose accept stream differs anywhere between two packed [n][words] arrays."""
    x = np.bitwise_or.reduce(np.bitwise_xor(got_words, want_words), axis=0)
    bits = np.unpackbits(x.view(np.uint8), bitorder="little")[:C]
    return np.flatnonzero(bits)


def run_gsn(state: OracleState, *, seed, rw_sigma, t_sigma, obs, iter0, nsteps, chain0=0, ll_mode=0, W=100,
            iters=None, history=True, nthreads=1, hist=None, accept_only=False):
    """Advance `state` by `nsteps` iterations of the single joint GaussianRW update.
    `hist` may be a preallocated alloc_history(C, D, nsteps) dict (reused buffers);
    accept_only: record the accept stream alone (hist["acc"] [nsteps][C])."""
    L = lib()
    Cn, D = state.C, state.D
    X = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, D))
    reuse = hist is not None
    if not reuse:
        hist = alloc_history(Cn, D, nsteps, accept_only) if (history or accept_only) else {}
    history = bool(hist)
    it = None
    if iters is not None:
        it = np.ascontiguousarray(iters, dtype=np.uint32)
    first = int(it[0]) if it is not None else int(iter0)
    if first > 1 and state.last_iter != first - 1:
        state.ra[:] = 0.0
    rc = L.orc_run_gsn(
        D, Cn, chain0, seed & 0xFFFFFFFFFFFFFFFF, _d(_colmajor(rw_sigma, D)), _d(_colmajor(t_sigma, D)), X.shape[0],
        _d(X), ll_mode, W, None if it is None else it.ctypes.data_as(C.POINTER(C.c_uint32)), iter0, nsteps,
        state.N, _d(state.theta), _d(state.ll), _d(state.ra), state.ring.ctypes.data_as(C.POINTER(C.c_uint64)),
        state.nacc.ctypes.data_as(C.POINTER(C.c_uint32)), state.faults.ctypes.data_as(C.POINTER(C.c_uint32)),
        _d(hist.get("theta")), _d(hist.get("prop")), _d(hist.get("ll")),
        None if not history else hist["acc"].ctypes.data_as(C.POINTER(C.c_uint8)), nthreads,
    )
    if rc != 0:
        raise ValueError(f"orc_run_gsn failed: {rc}")
    state.N += nsteps
    state.last_iter = int(it[-1]) if it is not None else int(iter0) + nsteps - 1
    if history and not reuse:
        hist["acc"] = hist["acc"].view(bool)  # 0/1 bytes: a view, no copy
    return hist


def cholesky(S):
    S = np.asarray(S, dtype=np.float64)
    D = S.shape[0]
    Lm = np.zeros(D * D)
    if lib().orc_cholesky(_d(_colmajor(S, D)), D, _d(Lm)) != 0:
        raise np.linalg.LinAlgError("not positive definite")
    return Lm.reshape(D, D)


def canon_sum(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().orc_canon_sum(_d(v), v.shape[0])


def gsn_constants(rw_sigma, t_sigma, obs):
    D = np.asarray(rw_sigma).shape[0]
    X = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, D))
    out = np.zeros(3 + D)
    Lr = np.zeros(D * D)
    Lt = np.zeros(D * D)
    rc = lib().orc_gsn_constants(D, _d(_colmajor(rw_sigma, D)), _d(_colmajor(t_sigma, D)), X.shape[0], _d(X),
                                 _d(out), _d(Lr), _d(Lt))
    if rc:
        raise ValueError(rc)
    return {"rw_c0": out[0], "t_c0": out[1], "S_c": out[2], "xbar": out[3:], "L_rw": Lr.reshape(D, D),
            "L_t": Lt.reshape(D, D)}


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    p = C.POINTER(C.c_uint32)
    lib().orc_philox(c.ctypes.data_as(p), k.ctypes.data_as(p), out.ctypes.data_as(p))
    return out


def step_variates(seed, chain, it, D, pidx0=0):
    """The D proposal normals and the accept Exp(1) draw of one (chain, iter)."""
    z = np.zeros(D)
    E = np.zeros(1)
    faults = lib().orc_step_variates(seed & 0xFFFFFFFFFFFFFFFF, chain, it, pidx0, D, _d(z), _d(E))
    return z, float(E[0]), int(faults)


def log_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_log_vec(_d(x), _d(y), x.size)
    return y


def exp_nonpos_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_exp_nonpos_vec(_d(x), _d(y), x.size)
    return y


def exp_any_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_exp_any_vec(_d(x), _d(y), x.size)
    return y


def exp_le0_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_exp_le0_vec(_d(x), _d(y), x.size)
    return y


def log_1_2_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_log_1_2_vec(_d(x), _d(y), x.size)
    return y


def rcp_1_2_vec(x):
    """1/u for u in [1, 2] as the MALA logistic terms form it (orc_log_rcp_1_2)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_rcp_1_2_vec(_d(x), _d(y), x.size)
    return y


def log_any_vec(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_log_any_vec(_d(x), _d(y), x.size)
    return y


def normals(seed, n, chain=0, iter0=1):
    out = np.empty(n)
    lib().orc_normal_vec(seed & 0xFFFFFFFFFFFFFFFF, chain, iter0, n, _d(out))
    return out


def exponentials(seed, n, chain0=0, it=1):
    out = np.empty(n)
    lib().orc_exp_vec(seed & 0xFFFFFFFFFFFFFFFF, chain0, it, n, _d(out))
    return out


ZIG_NORMAL_LAYERS = 8192  # oracle_math.h ORC_ZN_L


def zig_tables():
    """an[0..L+1] / fn[0..L+1]: normal strip edges x_j (an[L] = base width q)
    and f(x_j); ke/we/fe: the 256-strip Exp(1) table."""
    an, fn = np.empty(ZIG_NORMAL_LAYERS + 2), np.empty(ZIG_NORMAL_LAYERS + 2)
    ke = np.empty(256, dtype=np.uint64)
    we, fe = np.empty(256), np.empty(256)
    u64 = C.POINTER(C.c_uint64)
    lib().orc_zig_tables_copy(_d(an), _d(fn), ke.ctypes.data_as(u64), _d(we), _d(fe))
    return {"an": an, "fn": fn, "ke": ke, "we": we, "fe": fe}


def markstein_mismatches(b, x):
    """Count of x where the device's Markstein quotient differs from IEEE x / b."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    return int(lib().orc_markstein_mismatches(float(b), _d(x), x.size))


# ---- general schedule path (P ≥ 1 updates, Metropolis-within-Gibbs) ---------
MWG_MAXD = 64
KIND_UNIFORM, KIND_GAUSSIAN = 1, 2


PRIOR_IMPROPER, PRIOR_IMPROPER_POS, PRIOR_PRODUCT, PRIOR_STANDARD = 0, 1, 2, 3
DIST_NORMAL, DIST_UNIFORM, DIST_EXPONENTIAL, DIST_GAMMA = 1, 2, 3, 4
DIST_LOGNORMAL, DIST_BETA, DIST_INVERSE_GAMMA, DIST_CAUCHY, DIST_LAPLACE, DIST_TDIST = 5, 6, 7, 8, 9, 10
DIST_PRODUCT, DIST_MVNORMAL = 32, 33


KIND_USER = 5


KIND_MIX = 3
KIND_MALA = 4


def mwg_update(kind, coords0, eps=None, sigma=None, adapt=None, pos=None, prior=PRIOR_IMPROPER, factors=None,
               params=None, sigma_b=None, lam=0.5, haario_k=None):
    """One RandomWalkUpdate for run_mwg.  coords0: 0-based coordinates.
    adapt: None or dict(k, target, scale, min, max, offset) (AdaptationUnifRW).
    pos: None or per-coordinate positivity flags (UniformRandomWalk).
    prior: PRIOR_*; factors for PRIOR_PRODUCT / PRIOR_STANDARD, in constructor order, each
    (family, 1, a, b) for a univariate, (DIST_PRODUCT, k, [(family, a, b), ...]) for a
    Product of k univariates, (DIST_MVNORMAL, k, mu, Sigma) for an MvNormal; the count is
    the factor's `dims` entry (ProductPrior(dists, dims), priors.jl:64-79)."""
    return {"kind": kind, "coords": [int(c) for c in coords0], "eps": None if eps is None else list(eps),
            "sigma": None if sigma is None else np.asarray(sigma, dtype=np.float64), "adapt": adapt,
            "pos": None if pos is None else [bool(x) for x in pos], "prior": int(prior),
            "factors": [] if factors is None else [tuple(f) for f in factors],
            "params": None if params is None else [float(x) for x in np.ravel(params)],
            "sigma_b": None if sigma_b is None else np.asarray(sigma_b, dtype=np.float64), "lam": float(lam),
            "haario_k": haario_k}


class MWGState:
    """State of orc_run_mwg: the carried chain state and, for GaussianRandomWalkMix /
    HaarioTypeAdaptation updates and chain_moments, the per-chain L_B (from Σ_B),
    Haario mean/cov (zeros, N = 1 phantom sample) and GenericChainStats mean/cov."""

    def __init__(self, theta, mu0, updates, ll=None, chain_moments=False):
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        self.C, self.D = theta.shape
        P = len(updates)
        self.theta = theta.copy()
        self.mu_p = np.ascontiguousarray(np.broadcast_to(np.asarray(mu0, dtype=np.float64), theta.shape)).copy()
        self.ll = np.full(self.C, -np.inf) if ll is None else np.asarray(ll, dtype=np.float64).copy()
        self.ra = np.zeros((P, self.C))
        self.ring = np.zeros((P, self.C, 2), dtype=np.uint64)
        self.nacc = np.zeros((P, self.C), dtype=np.uint32)
        self.aprop = np.zeros((P, self.C), dtype=np.uint32)
        self.aacc = np.zeros((P, self.C), dtype=np.uint32)
        self.eps = np.zeros((P, self.C, MWG_MAXD))
        for p, u in enumerate(updates):
            if u["eps"] is not None:
                self.eps[p, :, :len(u["eps"])] = u["eps"]
        self.faults = np.zeros(self.C, dtype=np.uint32)
        self.N = np.array([1], dtype=np.uint64)
        self.last_iter = np.zeros(P, dtype=np.uint32)
        # mix / Haario / chain moments (the ext block of orc_run_mwg)
        ns = [len(u["coords"]) for u in updates]
        self.off_sq = np.array(np.cumsum([0] + [self.C * n * n for n in ns])[:P], dtype=np.uint64)
        self.off_v = np.array(np.cumsum([0] + [self.C * n for n in ns])[:P], dtype=np.uint64)
        tot_sq, tot_v = sum(self.C * n * n for n in ns), sum(self.C * n for n in ns)
        self.LB = np.zeros(tot_sq)
        self.hmean = np.zeros(tot_v)
        self.hcov = np.zeros(tot_sq)
        self.M = np.zeros(P, dtype=np.uint32)
        self.lam = np.array([float(u.get("lam", 0.0)) for u in updates])
        self.haario_k = np.array([int(u.get("haario_k") or 0) for u in updates], dtype=np.uint32)
        for p, u in enumerate(updates):
            if u["kind"] == 3:
                Lb = cholesky(np.asarray(u["sigma_b"], dtype=np.float64).reshape(ns[p], ns[p]))
                o = int(self.off_sq[p])
                self.LB[o:o + self.C * ns[p] ** 2] = np.tile(Lb.ravel(), self.C)
        self.chain_moments = bool(chain_moments)
        self.smean = np.zeros((self.C, self.D))
        self.scov = np.zeros((self.C, self.D, self.D))

    def lb(self, p, n):
        """The chains' L_B of update p: [C][n][n]."""
        o = int(self.off_sq[p])
        return self.LB[o:o + self.C * n * n].reshape(self.C, n, n)

    def haario(self, p, n):
        """The chains' Haario mean [C][n] and cov [C][n][n] of update p."""
        o, v = int(self.off_sq[p]), int(self.off_v[p])
        return (self.hmean[v:v + self.C * n].reshape(self.C, n),
                self.hcov[o:o + self.C * n * n].reshape(self.C, n, n))


class _MwgExt(C.Structure):
    """orc_mwg_ext (oracle/emcmc_oracle.c)."""
    _fields_ = [("mix_lam", C.POINTER(C.c_double)), ("haario_k", C.POINTER(C.c_uint32)),
                ("M_io", C.POINTER(C.c_uint32)), ("LB", C.POINTER(C.c_double)), ("hmean", C.POINTER(C.c_double)),
                ("hcov", C.POINTER(C.c_double)), ("off_sq", C.POINTER(C.c_uint64)),
                ("off_v", C.POINTER(C.c_uint64)), ("chain_moments", C.c_int), ("reserved", C.c_int),
                ("smean", C.POINTER(C.c_double)), ("scov", C.POINTER(C.c_double)), ("user_grad", C.c_void_p)]


def _mwg_tables(updates):
    P = len(updates)
    kind = np.zeros(P, dtype=np.uint32)
    nc = np.zeros(P, dtype=np.uint32)
    coords = np.zeros((P, MWG_MAXD), dtype=np.uint32)
    eps = np.zeros((P, MWG_MAXD))
    sigma = np.zeros((P, MWG_MAXD * MWG_MAXD))
    adapt = np.zeros(P, dtype=np.uint32)
    ak = np.ones(P, dtype=np.uint32)
    ap = np.zeros((P, 1 + 4 * MWG_MAXD))
    pos = np.zeros((P, MWG_MAXD), dtype=np.uint8)
    for p, u in enumerate(updates):
        n = len(u["coords"])
        kind[p], nc[p] = u["kind"], n
        coords[p, :n] = u["coords"]
        if u["eps"] is not None:
            eps[p, :n] = u["eps"]
        if u["sigma"] is not None:
            sigma[p, :n * n] = np.asarray(u["sigma"], dtype=np.float64).reshape(n, n).ravel(order="F")
        if u["adapt"] is not None:
            a = u["adapt"]
            adapt[p], ak[p] = 1, a["k"]
            ap[p, 0] = a["target"]
            for f, name in enumerate(("scale", "min", "max", "offset")):  # per coordinate (scalars repeat)
                v = np.atleast_1d(np.asarray(a[name], dtype=np.float64))
                row = ap[p, 1 + f * MWG_MAXD: 1 + (f + 1) * MWG_MAXD]
                row[:] = v[0]
                row[:v.size] = v
        if u.get("pos") is not None:
            pos[p, :n] = np.asarray(u["pos"], dtype=bool)
    return kind, nc, coords, eps, sigma, adapt, ak, ap, pos


def _prior_tables(updates):
    """Flat prior tables of orc_run_mwg: factors (ffam, fcnt, fa, fb), Product
    components (cfam, ca, cb, consecutively in factor order) and MvNormal μ / Σ
    placed at the local range the factor reads (the constructor's `last`)."""
    P = len(updates)
    pk = np.zeros(P, dtype=np.uint32)
    nf = np.zeros(P, dtype=np.uint32)
    ffam = np.zeros((P, MWG_MAXD), dtype=np.uint32)
    fcnt = np.zeros((P, MWG_MAXD), dtype=np.uint32)
    fa = np.zeros((P, MWG_MAXD))
    fb = np.zeros((P, MWG_MAXD))
    cfam = np.zeros((P, MWG_MAXD), dtype=np.uint32)
    ca = np.zeros((P, MWG_MAXD))
    cb = np.zeros((P, MWG_MAXD))
    mvmu = np.zeros((P, MWG_MAXD))
    mvS = np.zeros((P, MWG_MAXD, MWG_MAXD))  # [p][col][row]: column-major 64 × 64 blocks
    for p, u in enumerate(updates):
        pk[p] = u.get("prior", PRIOR_IMPROPER)
        fs = u.get("factors", [])
        nf[p] = len(fs)
        last, nc = 0, 0
        for k, f in enumerate(fs):
            fam, cnt = int(f[0]), int(f[1])
            ffam[p, k], fcnt[p, k] = fam, cnt
            st = 0 if cnt == 1 else last
            last += cnt
            if fam == DIST_PRODUCT:
                for (cf, a, b) in f[2]:
                    cfam[p, nc], ca[p, nc], cb[p, nc] = cf, a, b
                    nc += 1
            elif fam == DIST_MVNORMAL:
                mu = np.asarray(f[2], dtype=np.float64).reshape(cnt)
                S = np.asarray(f[3], dtype=np.float64).reshape(cnt, cnt)
                mvmu[p, st:st + cnt] = mu
                mvS[p, st:st + cnt, st:st + cnt] = S.T  # [col][row]
            else:
                fa[p, k], fb[p, k] = f[2], f[3]
    return pk, nf, ffam, fcnt, fa, fb, cfam, ca, cb, mvmu, mvS


def eval_prior(prior, n, factors, x):
    """logpdf(prior, x) of one update's prior (orc_eval_prior) at each row of x
    ([m][n]); factors as in mwg_update.  Raises ValueError with the oracle's
    status (−2 invalid, −4 a pairing the reference raises a MethodError on)."""
    L = lib()
    if not hasattr(L, "_evp_ready"):
        dp, u32p = C.POINTER(C.c_double), C.POINTER(C.c_uint32)
        L.orc_eval_prior.restype = C.c_int
        L.orc_eval_prior.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p, dp, dp, u32p, dp, dp, dp, dp,
                                     C.c_uint64, dp, dp]
        L._evp_ready = True
    pk, nf, ffam, fcnt, fa, fb, cfam, ca, cb, mvmu, mvS = _prior_tables([{"prior": prior, "factors": factors or []}])
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1, n))
    out = np.empty(x.shape[0])
    u32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
    rc = L.orc_eval_prior(int(prior), n, int(nf[0]), u32(ffam), u32(fcnt), _d(fa), _d(fb), u32(cfam), _d(ca),
                          _d(cb), _d(mvmu), _d(mvS), x.shape[0], _d(x), _d(out))
    if rc != 0:
        raise ValueError(f"orc_eval_prior: {rc}")
    return out


USER_LL_FN = C.CFUNCTYPE(C.c_double, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double), C.c_uint64,
                         C.POINTER(C.c_double))


def run_mwg(state: MWGState, updates, *, seed, t_sigma, obs, steps, chain0=0, ll_mode=0, W=100, history=True,
            nthreads=1, user_ll=None, user_params=None, user_upd=None, user_grad=None):
    """Advance `state` over `steps` [(mcmciter, pidx 1-based), …]; histories per step.
    user_ll: a C function pointer (ctypes) of the user target's loglikelihood, or None
    for GsnTargetLaw; user_grad: the law's EMCMC_USER_GRAD (MALA updates, kind 4, on a user
    law); state.ll_prop receives sub_ws°.ll of every update."""
    L = lib()
    if not hasattr(L, "_mwg_ready"):
        dp, u32p, u64p, u8p = (C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                               C.POINTER(C.c_uint8))
        L.orc_run_mwg.restype = C.c_int
        L.orc_run_mwg.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, u32p, u32p, u32p, dp, dp,
                                  u8p, u32p, u32p, dp, dp, C.c_uint64, dp, C.c_int, C.c_uint32, C.c_uint32, u32p, u32p,
                                  u64p, u32p, dp, dp, dp, dp, u64p, u32p, u32p, u32p, dp, u32p, dp, dp, dp, u8p,
                                  C.c_int, u32p, u32p, u32p, u32p, dp, dp, dp, C.c_void_p, dp, u32p, dp, dp, dp, dp,
                                  C.c_void_p, C.c_void_p, dp, C.POINTER(_MwgExt)]
        L._mwg_ready = True
    Cn, D = state.C, state.D
    kind, nc, coords, eps, sigma, adapt, ak, ap, pos = _mwg_tables(updates)
    pk, nf, ffam, fcnt, fa, fb, cfam, ca, cb, mvmu, mvS = _prior_tables(updates)
    uparams = np.zeros((len(updates), MWG_MAXD * MWG_MAXD))  # user updates: their parameters
    for p, u in enumerate(updates):
        if u.get("params") is not None:
            v = np.asarray(u["params"], dtype=np.float64).ravel()
            uparams[p, :v.size] = v
    if getattr(state, "ll_prop", None) is None:
        state.ll_prop = np.full((len(updates), state.C), np.nan)
    state.lam = np.ascontiguousarray(state.lam, dtype=np.float64)
    ext = _MwgExt(_d(state.lam), state.haario_k.ctypes.data_as(C.POINTER(C.c_uint32)),
                  state.M.ctypes.data_as(C.POINTER(C.c_uint32)), _d(state.LB), _d(state.hmean), _d(state.hcov),
                  state.off_sq.ctypes.data_as(C.POINTER(C.c_uint64)),
                  state.off_v.ctypes.data_as(C.POINTER(C.c_uint64)), int(state.chain_moments), 0, _d(state.smean),
                  _d(state.scov), None if user_grad is None else C.cast(user_grad, C.c_void_p))
    up = None if user_params is None else np.ascontiguousarray(user_params, dtype=np.float64)
    steps = np.asarray(steps, dtype=np.uint32).reshape(-1, 2)
    si = np.ascontiguousarray(steps[:, 0])
    sp = np.ascontiguousarray(steps[:, 1])
    n = steps.shape[0]
    if user_ll is None:
        X = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, D))
    else:  # a user law's observation rows have their own width
        X = np.zeros((0, 1)) if obs is None else np.asarray(obs, dtype=np.float64)
        X = np.ascontiguousarray(X.reshape(X.shape[0], max(1, int(np.prod(X.shape[1:])))) if X.ndim > 1 else X.reshape(-1, 1))
        if t_sigma is None:
            t_sigma = np.eye(D)
    hist = {"theta": np.empty((n, Cn, D)), "prop": np.empty((n, Cn, D)), "ll": np.empty((n, Cn)),
            "acc": np.empty((n, Cn), dtype=np.uint8)} if history else {}
    u32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
    u64 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint64))  # noqa: E731
    rc = L.orc_run_mwg(
        D, Cn, chain0, seed & 0xFFFFFFFFFFFFFFFF, len(updates), u32(kind), u32(nc), u32(coords), _d(eps), _d(sigma),
        pos.ctypes.data_as(C.POINTER(C.c_uint8)), u32(adapt), u32(ak), _d(ap), _d(_colmajor(t_sigma, D)), X.shape[0], _d(X), ll_mode, W, n, u32(si), u32(sp),
        u64(state.N), u32(state.last_iter), _d(state.theta), _d(state.mu_p), _d(state.ll), _d(state.ra),
        u64(state.ring), u32(state.nacc), u32(state.aprop), u32(state.aacc), _d(state.eps), u32(state.faults),
        _d(hist.get("theta")), _d(hist.get("prop")), _d(hist.get("ll")),
        None if not history else hist["acc"].ctypes.data_as(C.POINTER(C.c_uint8)), nthreads,
        u32(pk), u32(nf), u32(ffam), u32(fcnt), _d(fa), _d(fb), _d(state.ll_prop),
        None if user_ll is None else C.cast(user_ll, C.c_void_p), None if up is None else _d(up),
        u32(cfam), _d(ca), _d(cb), _d(mvmu), _d(mvS),
        None if user_upd is None else C.cast(user_upd[0], C.c_void_p),
        None if user_upd is None else C.cast(user_upd[1], C.c_void_p), _d(uparams), C.byref(ext))
    if rc != 0:
        raise ValueError(f"orc_run_mwg failed: {rc}")
    if history:
        hist["acc"] = hist["acc"].astype(bool)
    return hist


def user_loglik(name):
    """The oracle build of user target tests/user_targets/<name>.c or of a law the
    library ships, extensiblemcmc.jl_amd/csrc/laws/<name>.c (oracle/Makefile:
    lib/user_<name>.so, compiled with oracle/user_prelude.h): (ctypes function,
    source text).  The engine compiles the same source for the device."""
    so = Path(__file__).resolve().parent / "lib" / f"user_{name}.so"
    root = Path(__file__).resolve().parent.parent
    src = root / "tests" / "user_targets" / f"{name}.c"
    if not src.exists():
        src = root / "extensiblemcmc.jl_amd" / "csrc" / "laws" / f"{name}.c"
    if not so.exists():
        raise ImportError(f"{so} not built (make -C oracle)")
    dll = C.CDLL(str(so))
    fn = USER_LL_FN(("emcmc_user_loglik", dll))
    fn._dll = dll  # keep the library loaded
    return fn, src.read_text()


USER_GRAD_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double), C.c_uint64,
                           C.POINTER(C.c_double), C.POINTER(C.c_double))


def user_grad(name):
    """The oracle build's emcmc_user_grad of user target tests/user_targets/<name>.c
    (a law whose source defines EMCMC_USER_GRAD), as a ctypes function."""
    so = Path(__file__).resolve().parent / "lib" / f"user_{name}.so"
    if not so.exists():
        raise ImportError(f"{so} not built (make -C oracle)")
    dll = C.CDLL(str(so))
    fn = USER_GRAD_FN(("emcmc_user_grad", dll))
    fn._dll = dll
    return fn


USER_PROP_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double),
                           C.c_void_p)
USER_LTD_FN = C.CFUNCTYPE(C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double))


def user_update(name):
    """The oracle build of user update tests/user_updates/<name>.c (oracle/Makefile:
    lib/userupd_<name>.so, compiled with oracle/user_prelude.h): ((proposal, ltd)
    ctypes functions, source text).  The engine compiles the same source for the device."""
    so = Path(__file__).resolve().parent / "lib" / f"userupd_{name}.so"
    src = Path(__file__).resolve().parent.parent / "tests" / "user_updates" / f"{name}.c"
    if not so.exists():
        raise ImportError(f"{so} not built (make -C oracle)")
    dll = C.CDLL(str(so))
    prop = USER_PROP_FN(("emcmc_user_proposal", dll))
    ltd = USER_LTD_FN(("emcmc_user_ltd", dll))
    prop._dll = ltd._dll = dll
    return (prop, ltd), src.read_text()


def uniform01(seed, chain, it, pidx0, j):
    """The [0,1) uniform of coordinate j (update-local) of a UniformRandomWalk draw."""
    r = philox([chain, it, j >> 1, (pidx0 << 16)], [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF])
    hi, lo = (int(r[2]), int(r[3])) if j & 1 else (int(r[0]), int(r[1]))
    return float((hi << 21) | (lo >> 11)) * 2.0 ** -53


# ---- GaussianRandomWalkMix + HaarioTypeAdaptation + chain moments (cfg 4) ---
class MixState(OracleState):
    """OracleState plus GenericChainStats mean/cov (phantom zero sample: N = 1,
    mean = 0, cov = 0), the per-chain Cholesky factor L_B of Σ_B and Haario's M."""

    def __init__(self, theta, sigma_b=None, ll=None):
        super().__init__(theta, ll)
        D = self.D
        self.mean = np.zeros((self.C, D))
        self.cov = np.zeros((self.C, D, D))
        LB = cholesky(sigma_b) if sigma_b is not None else np.eye(D)
        self.LB = np.ascontiguousarray(np.broadcast_to(LB, (self.C, D, D))).copy()
        self.M = 0


def run_mix(state: MixState, *, seed, sigma_a, t_sigma, obs, iter0, nsteps, mix=True, lam=0.5, haario_k=0,
            chain0=0, ll_mode=0, W=100, history=True, nthreads=1, accept_only=False):
    """Advance `state` by `nsteps` consecutive iterations of the single joint
    GaussianRandomWalkMix (mix=True) or GaussianRandomWalk (mix=False) update
    with on-device chain moments; haario_k > 0 adds HaarioTypeAdaptation(k).
    accept_only: record the accept stream alone (hist["acc"] [nsteps][C])."""
    L = lib()
    if not hasattr(L, "_mix_ready"):
        dp, u32p, u64p, u8p = (C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                               C.POINTER(C.c_uint8))
        L.orc_run_mix.restype = C.c_int
        L.orc_run_mix.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, dp, C.c_int, C.c_double, C.c_int,
                                  C.c_uint32, dp, C.c_uint64, dp, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, u64p,
                                  u32p, dp, dp, dp, u64p, u32p, u32p, dp, dp, dp, dp, dp, dp, u8p, C.c_int]
        L._mix_ready = True
    Cn, D = state.C, state.D
    X = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, D))
    hist = alloc_history(Cn, D, nsteps, accept_only) if (history or accept_only) else {}
    history = bool(hist)
    if iter0 > 1 and state.last_iter != iter0 - 1:
        state.ra[:] = 0.0
    N = np.array([state.N], dtype=np.uint64)
    M = np.array([state.M], dtype=np.uint32)
    rc = L.orc_run_mix(
        D, Cn, chain0, seed & 0xFFFFFFFFFFFFFFFF, _d(_colmajor(sigma_a, D)), int(mix), float(lam),
        int(haario_k > 0), max(int(haario_k), 1), _d(_colmajor(t_sigma, D)), X.shape[0], _d(X), ll_mode, W, iter0,
        nsteps, N.ctypes.data_as(C.POINTER(C.c_uint64)), M.ctypes.data_as(C.POINTER(C.c_uint32)), _d(state.theta),
        _d(state.ll), _d(state.ra), state.ring.ctypes.data_as(C.POINTER(C.c_uint64)),
        state.nacc.ctypes.data_as(C.POINTER(C.c_uint32)), state.faults.ctypes.data_as(C.POINTER(C.c_uint32)),
        _d(state.mean), _d(state.cov), _d(state.LB), _d(hist.get("theta")), _d(hist.get("prop")),
        _d(hist.get("ll")), None if not history else hist["acc"].ctypes.data_as(C.POINTER(C.c_uint8)), nthreads)
    if rc != 0:
        raise ValueError(f"orc_run_mix failed: {rc}")
    state.N, state.M = int(N[0]), int(M[0])
    state.last_iter = iter0 + nsteps - 1
    if history:
        hist["acc"] = hist["acc"].view(bool)
    return hist


def pick_uniform(seed, chain, it, pidx0=0, attempt=0):
    """The [0,1) uniform that picks GaussianRandomWalkMix's kernel (B iff u ≤ λ):
    block 0xFFFFFFFE of (chain, iter), update pidx0, redraw `attempt`."""
    r = philox([chain, it, 0xFFFFFFFE, (pidx0 << 16) | attempt], [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF])
    return float((int(r[0]) << 21) | (int(r[1]) >> 11)) * 2.0 ** -53


# ---- MALA on a logistic-regression target (row f2, cfg 3) -------------------
def _mala_sigs(L):
    if not hasattr(L, "_mala_ready"):
        dp, u32p, u64p, u8p = (C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                               C.POINTER(C.c_uint8))
        L.orc_logistic_eval_batch.restype = None
        L.orc_logistic_eval_batch.argtypes = [C.c_int, C.c_uint64, dp, dp, C.c_uint64, dp, dp, dp, C.c_int]
        L.orc_run_mala.restype = C.c_int
        L.orc_run_mala.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_double, dp, dp, C.c_uint64,
                                   C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, dp, dp, dp, dp, u64p, u32p, u32p,
                                   dp, dp, dp, u8p, C.c_int]
        L._mala_ready = True


def logistic_eval(X, y, theta, nthreads=1):
    """ℓ [C] and ∇ℓ [C][D] at theta [C][D] (the engine's evaluation order)."""
    L = lib()
    _mala_sigs(L)
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    th = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    Cn, D = th.shape
    ll = np.empty(Cn)
    g = np.empty((Cn, D))
    L.orc_logistic_eval_batch(D, Cn, _d(X), _d(y), X.shape[0], _d(th), _d(ll), _d(g), nthreads)
    return ll, g


class MALAState(OracleState):
    """OracleState plus the carried gradient ∇ℓ(θ), evaluated at θinit."""

    def __init__(self, theta, X, y, ll=None, nthreads=1):
        super().__init__(theta, ll)
        _, self.grad = logistic_eval(X, y, self.theta, nthreads)


def run_mala(state: MALAState, *, seed, eps, X, y, iter0, nsteps, chain0=0, W=100, history=True, nthreads=1):
    L = lib()
    _mala_sigs(L)
    Cn, D = state.C, state.D
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    hist = alloc_history(Cn, D, nsteps) if history else {}
    if iter0 > 1 and state.last_iter != iter0 - 1:
        state.ra[:] = 0.0
    rc = L.orc_run_mala(D, Cn, chain0, seed & 0xFFFFFFFFFFFFFFFF, float(eps), _d(X), _d(y), X.shape[0], W, iter0,
                        nsteps, state.N, _d(state.theta), _d(state.grad), _d(state.ll), _d(state.ra),
                        state.ring.ctypes.data_as(C.POINTER(C.c_uint64)),
                        state.nacc.ctypes.data_as(C.POINTER(C.c_uint32)),
                        state.faults.ctypes.data_as(C.POINTER(C.c_uint32)), _d(hist.get("theta")),
                        _d(hist.get("prop")), _d(hist.get("ll")),
                        None if not history else hist["acc"].ctypes.data_as(C.POINTER(C.c_uint8)), nthreads)
    if rc != 0:
        raise ValueError(f"orc_run_mala failed: {rc}")
    state.N += nsteps
    state.last_iter = iter0 + nsteps - 1
    if history:
        hist["acc"] = hist["acc"].astype(bool)
    return hist
