"""Thin object wrapper over one ``emcmc_handle`` (one shard of chains on one GPU).

Every method is a direct call through the C ABI (include/emcmc.h); nothing here
computes on the host beyond packing arguments.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


@dataclass
class EngineConfig:
    dim: int
    num_chains: int
    num_mcmc_steps: int
    seed: int = 0
    first_chain_id: int = 0
    device: int = 0
    history_mode: int = L.HIST_FULL
    roll_window: int = 100
    lanes_per_chain: int = 0
    steps_per_launch: int = 0
    kernel_variant: int = 0
    chain_moments: bool = False
    history_ring: int = 0  # iterations of history kept on device (0 = all)


class PinnedArray(np.ndarray):
    """A numpy array over page-locked host memory (emcmc_host_alloc); the memory
    is released when the array (and every view of it) is garbage collected."""

    def __new__(cls, shape, dtype):
        dt = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dt.itemsize
        p = C.c_void_p()
        st = L.lib().emcmc_host_alloc(max(1, nbytes), C.byref(p))
        if st != L.OK:
            raise L.EMCMCError(st, "emcmc_host_alloc")
        buf = (C.c_char * max(1, nbytes)).from_address(p.value)
        obj = np.ndarray.__new__(cls, shape, dtype=dt, buffer=buf)
        obj._owner = _PinnedOwner(p.value)
        return obj

    def __array_finalize__(self, obj):
        if obj is not None and not hasattr(self, "_owner"):
            self._owner = getattr(obj, "_owner", None)


class _PinnedOwner:
    def __init__(self, addr):
        self.addr = addr

    def __del__(self):
        try:
            L.lib().emcmc_host_free(C.c_void_p(self.addr))
        except Exception:
            pass


class Engine:
    def __init__(self, cfg: EngineConfig):
        self.cfg = cfg
        self._lib = L.lib()
        L.check_single_hip_runtime()  # warns once if torch's runtime was mapped beside the library's
        self._run_memo = None
        c = L.EmcmcConfig()
        c.abi_version = L.ABI_VERSION
        c.dim = cfg.dim
        c.num_chains = cfg.num_chains
        c.first_chain_id = cfg.first_chain_id
        c.num_mcmc_steps = cfg.num_mcmc_steps
        c.seed = cfg.seed & 0xFFFFFFFFFFFFFFFF
        c.device = cfg.device
        c.history_mode = cfg.history_mode
        c.roll_window = cfg.roll_window
        c.lanes_per_chain = cfg.lanes_per_chain
        c.steps_per_launch = cfg.steps_per_launch
        c.kernel_variant = cfg.kernel_variant
        c.chain_moments = int(bool(cfg.chain_moments))
        c.history_ring = int(cfg.history_ring)
        h = C.c_void_p()
        st = self._lib.emcmc_create(C.byref(h), C.byref(c))
        if st != L.OK:
            raise L.EMCMCError(st, "emcmc_create", "" if st != L.NO_DEVICE else "no HIP device visible")
        self._h = h
        self.num_updates = 0
        self._update_n = []  # coordinates per update (shapes of per-update read-backs)
        self._cb_error = None  # an exception raised inside a host callback (fλ), re-raised after emcmc_run

    # -- plumbing -------------------------------------------------------------
    def _check(self, st: int, where: str):
        if st != L.OK:
            msg = self._lib.emcmc_last_error(self._h)
            cls = L.UnsupportedPluginError if st == L.UNSUPPORTED_PLUGIN else L.EMCMCError
            raise cls(st, where, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.emcmc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- setup ------------------------------------------------------------------
    @staticmethod
    def _prior_factor(f, keep):
        """One emcmc_prior_factor from (family, 1, a, b), (DIST_PRODUCT, k, [(family, a, b), ...])
        or (DIST_MVNORMAL, k, mu, Sigma) — count is the factor's dims entry."""
        fam, cnt = int(f[0]), int(f[1])
        pf = L.EmcmcPriorFactor()
        pf.family, pf.count = fam, cnt
        if fam == L.DIST_PRODUCT:
            comps = (L.EmcmcPriorFactor * len(f[2]))()
            for i, (cf, a, b) in enumerate(f[2]):
                comps[i].family, comps[i].count, comps[i].a, comps[i].b = int(cf), 1, float(a), float(b)
            keep.append(comps)
            pf.components = C.cast(comps, C.POINTER(L.EmcmcPriorFactor))
        elif fam == L.DIST_MVNORMAL:
            mu = np.ascontiguousarray(np.asarray(f[2], dtype=np.float64).reshape(cnt))
            S = np.ascontiguousarray(np.asarray(f[3], dtype=np.float64).reshape(cnt, cnt).ravel(order="F"))
            keep += [mu, S]
            pf.mu = mu.ctypes.data_as(C.POINTER(C.c_double))
            pf.sigma = S.ctypes.data_as(C.POINTER(C.c_double))
        else:
            pf.a, pf.b = float(f[2]), float(f[3])
        return pf

    @classmethod
    def _prior_desc(cls, u, prior, factors, keep):
        """emcmc_update_desc.prior/prior_params; factors in constructor order (_prior_factor)."""
        u.prior = prior
        if factors:
            arr = (L.EmcmcPriorFactor * len(factors))(*[cls._prior_factor(f, keep) for f in factors])
            pd = L.EmcmcPriorDesc(len(factors), 0, C.cast(arr, C.POINTER(L.EmcmcPriorFactor)))
            keep += [arr, pd]
            u.prior_params = C.cast(C.pointer(pd), C.c_void_p)

    @classmethod
    def gaussian_rw_desc(cls, coords0, sigma, prior=L.PRIOR_IMPROPER, adaptation=L.ADPT_NONE, pos=None,
                         prior_factors=None):
        """(emcmc_update_desc, keepalive) of GaussianRandomWalk(Σ) on coords0 (0-based)."""
        keep = []
        coords = np.ascontiguousarray(coords0, dtype=np.uint32)
        S = np.asfortranarray(np.asarray(sigma, dtype=np.float64).reshape(len(coords), len(coords)))
        Sf = np.ascontiguousarray(S.ravel(order="F"))
        keep += [coords, Sf]
        u = L.EmcmcUpdateDesc()
        u.kernel = L.RW_GAUSSIAN
        cls._prior_desc(u, prior, prior_factors, keep)
        u.adaptation = adaptation
        u.num_coords = len(coords)
        u.coords = L.u32ptr(coords)
        u.sigma = L.dptr(Sf)
        if pos is not None:
            p = np.ascontiguousarray(pos, dtype=np.uint8)
            keep.append(p)
            u.pos = p.ctypes.data_as(C.POINTER(C.c_uint8))
        return u, keep

    def add_gaussian_rw_update(self, coords0, sigma, prior=L.PRIOR_IMPROPER, adaptation=L.ADPT_NONE, pos=None,
                               prior_factors=None):
        u, keep = self.gaussian_rw_desc(coords0, sigma, prior, adaptation, pos, prior_factors)
        self.add_update_desc(u, keep)

    @classmethod
    def uniform_rw_desc(cls, coords0, eps, adapt=None, prior=L.PRIOR_IMPROPER, pos=None, prior_factors=None):
        """(emcmc_update_desc, keepalive) of UniformRandomWalk(ϵ) on coords0 (0-based); adapt: None
        or a dict with AdaptationUnifRW's k, target, scale, min, max, offset."""
        keep = []
        coords = np.ascontiguousarray(coords0, dtype=np.uint32)
        e = np.ascontiguousarray(np.broadcast_to(np.asarray(eps, dtype=np.float64), (len(coords),)))
        keep += [coords, e]
        u = L.EmcmcUpdateDesc()
        u.kernel = L.RW_UNIFORM
        cls._prior_desc(u, prior, prior_factors, keep)
        u.num_coords = len(coords)
        u.coords = L.u32ptr(coords)
        u.epsilon = L.dptr(e)
        ad = None
        if adapt is not None:
            names = ("scale", "min", "max", "offset")
            if all(np.ndim(adapt[k]) == 0 for k in names):
                ad = L.EmcmcUnifRWAdaptation(int(adapt["k"]), 0, float(adapt["target"]), float(adapt["scale"]),
                                             float(adapt["min"]), float(adapt["max"]), float(adapt["offset"]))
                u.adaptation = L.ADPT_UNIF_RW
            else:  # per-coordinate form (adaptation.jl:155-188)
                arrs = [np.ascontiguousarray(np.broadcast_to(np.asarray(adapt[k], dtype=np.float64),
                                                             (len(coords),))) for k in names]
                keep.extend(arrs)
                ad = L.EmcmcUnifRWAdaptationVec(int(adapt["k"]), 0, float(adapt["target"]),
                                                *[L.dptr(a) for a in arrs])
                u.adaptation = L.ADPT_UNIF_RW_VEC
            keep.append(ad)
            u.adaptation_params = C.cast(C.pointer(ad), C.c_void_p)
        if pos is not None:
            p = np.ascontiguousarray(pos, dtype=np.uint8)
            keep.append(p)
            u.pos = p.ctypes.data_as(C.POINTER(C.c_uint8))
        return u, keep

    def add_uniform_rw_update(self, coords0, eps, adapt=None, prior=L.PRIOR_IMPROPER, pos=None, prior_factors=None):
        """UniformRandomWalk(ϵ) on coords0 (0-based); adapt: None or a dict with
        AdaptationUnifRW's k, target, scale, min, max, offset."""
        u, keep = self.uniform_rw_desc(coords0, eps, adapt, prior, pos, prior_factors)
        self.add_update_desc(u, keep)

    def add_gaussian_rw_mix_update(self, coords0, sigma_a, sigma_b, lam=0.5, haario_k=None, haario_scale=2.38 ** 2,
                                   prior=L.PRIOR_IMPROPER, pos=None, prior_factors=None):
        """GaussianRandomWalkMix(Σ_A, Σ_B, λ) on coords0 (0-based); haario_k: None
        or HaarioTypeAdaptation's adapt_every_k_steps."""
        coords = np.ascontiguousarray(coords0, dtype=np.uint32)
        n = len(coords)
        SA = np.ascontiguousarray(np.asarray(sigma_a, dtype=np.float64).reshape(n, n).ravel(order="F"))
        SB = np.ascontiguousarray(np.asarray(sigma_b, dtype=np.float64).reshape(n, n).ravel(order="F"))
        keep = []
        u = L.EmcmcUpdateDesc()
        u.kernel = L.RW_GAUSSIAN_MIX
        self._prior_desc(u, prior, prior_factors, keep)
        u.num_coords = n
        u.coords = L.u32ptr(coords)
        u.sigma = L.dptr(SA)
        u.sigma_b = L.dptr(SB)
        u.mix_lambda = float(lam)
        ad = None
        if haario_k is not None:
            ad = L.EmcmcHaarioAdaptation(int(haario_k), 0, float(haario_scale))
            u.adaptation = L.ADPT_HAARIO
            u.adaptation_params = C.cast(C.pointer(ad), C.c_void_p)
        if pos is not None:
            p = np.ascontiguousarray(pos, dtype=np.uint8)
            u.pos = p.ctypes.data_as(C.POINTER(C.c_uint8))
        self._check(self._lib.emcmc_add_update(self._h, C.byref(u)), "emcmc_add_update")
        self.num_updates += 1
        self._update_n.append(int(len(coords)))

    def add_user_update(self, coords0, source, params=(), options="", prior=L.PRIOR_IMPROPER, prior_factors=None):
        """A user-defined update on coords0 (0-based): its proposal! and
        log_transition_density as an EMCMC_USER_PROPOSAL / EMCMC_USER_LTD source
        (include/emcmc.h emcmc_user_update_desc; updates.jl:42-93), compiled at run time."""
        keep = []
        coords = np.ascontiguousarray(coords0, dtype=np.uint32)
        prm = np.ascontiguousarray(np.ravel(np.asarray(params, dtype=np.float64)))
        ud = L.EmcmcUserUpdateDesc(source.encode(), options.encode() if options else None, prm.size,
                                   L.dptr(prm) if prm.size else None)
        keep += [prm, ud]
        u = L.EmcmcUpdateDesc()
        u.kernel = L.USER_UPDATE
        self._prior_desc(u, prior, prior_factors, keep)
        u.num_coords = len(coords)
        u.coords = L.u32ptr(coords)
        u.user_update = C.cast(C.pointer(ud), C.c_void_p)
        self._check(self._lib.emcmc_add_update(self._h, C.byref(u)), "emcmc_add_update")
        self.num_updates += 1
        self._update_n.append(int(len(coords)))

    def add_mala_update(self, coords0, eps, prior=L.PRIOR_IMPROPER, prior_factors=None):
        """MALA with step size ϵ on coords0 (0-based; the engine's definition of
        the reference's stub MALAUpdate, updates.jl:216-218).  On the logistic
        target: the fused MFMA kernel (one joint update, ImproperPrior); on
        GsnTargetLaw or a user law with EMCMC_USER_GRAD: the general kernel (any
        coordinates, any prior, beside other updates)."""
        keep = []
        coords = np.ascontiguousarray(coords0, dtype=np.uint32)
        e = np.array([float(eps)])
        u = L.EmcmcUpdateDesc()
        u.kernel = L.MALA
        self._prior_desc(u, prior, prior_factors, keep)
        u.num_coords = len(coords)
        u.coords = L.u32ptr(coords)
        u.epsilon = L.dptr(e)
        self._check(self._lib.emcmc_add_update(self._h, C.byref(u)), "emcmc_add_update")
        self.num_updates += 1
        self._update_n.append(int(len(coords)))

    def set_logistic_target(self, X, y):
        """Logistic regression: ℓ(θ) = Σ_n y_n x_nᵀθ − log(1 + exp(x_nᵀθ))."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        yv = np.ascontiguousarray(y, dtype=np.float64).reshape(X.shape[0])
        t = L.EmcmcTargetDesc()
        t.kind = L.TARGET_LOGISTIC
        t.dim = X.shape[1]
        t.num_obs = X.shape[0]
        t.obs = L.dptr(X)
        t.labels = L.dptr(yv)
        self._check(self._lib.emcmc_set_target(self._h, C.byref(t)), "emcmc_set_target")

    def add_update_desc(self, u: L.EmcmcUpdateDesc, keepalive=()):
        self._check(self._lib.emcmc_add_update(self._h, C.byref(u)), "emcmc_add_update")
        self.num_updates += 1
        self._update_n.append(int(u.num_coords))

    def set_gsn_target(self, mu, sigma, obs, ll_mode=L.LL_PER_OBS):
        mu = np.ascontiguousarray(mu, dtype=np.float64)
        d = mu.shape[0]
        Sf = np.ascontiguousarray(np.asarray(sigma, dtype=np.float64).reshape(d, d).ravel(order="F"))
        X = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, d))
        t = L.EmcmcTargetDesc()
        t.kind = L.TARGET_GSN
        t.dim = d
        t.mu = L.dptr(mu)
        t.sigma = L.dptr(Sf)
        t.num_obs = X.shape[0]
        t.obs = L.dptr(X)
        t.ll_mode = ll_mode
        self._check(self._lib.emcmc_set_target(self._h, C.byref(t)), "emcmc_set_target")

    def set_user_target(self, source: str, obs=None, params=None, theta0=None, options: str = ""):
        """A user law: ``loglikelihood(P, obs)`` as an EMCMC_USER_LOGLIK source
        compiled for the device (include/emcmc.h emcmc_user_target_desc)."""
        D = self.cfg.dim
        X = np.zeros((0, 1)) if obs is None else np.asarray(obs, dtype=np.float64)
        X = np.ascontiguousarray(X.reshape(X.shape[0], max(1, int(np.prod(X.shape[1:])))) if X.ndim > 1 else X.reshape(-1, 1))
        prm = np.ascontiguousarray(np.zeros(0) if params is None else np.asarray(params, dtype=np.float64).ravel())
        th0 = np.ascontiguousarray(np.zeros(D) if theta0 is None else np.asarray(theta0, dtype=np.float64).ravel())
        t = L.EmcmcUserTargetDesc()
        t.dim = D
        t.obs_dim = X.shape[1]
        t.theta0 = L.dptr(th0)
        t.num_obs = X.shape[0]
        t.obs = L.dptr(X) if X.size else None
        t.num_params = prm.size
        t.params = L.dptr(prm) if prm.size else None
        t.source = source.encode()
        t.options = options.encode()
        self._check(self._lib.emcmc_set_user_target(self._h, C.byref(t)), "emcmc_set_user_target")

    def set_state(self, theta, ll=None):
        th = np.ascontiguousarray(theta, dtype=np.float64).reshape(self.cfg.num_chains, self.cfg.dim)
        llp = None
        if ll is not None:
            la = np.ascontiguousarray(ll, dtype=np.float64).reshape(self.cfg.num_chains)
            llp = L.dptr(la)
        self._check(self._lib.emcmc_set_state(self._h, L.dptr(th), llp), "emcmc_set_state")

    # -- run ----------------------------------------------------------------------
    def run(self, steps):
        """steps: iterable of (mcmciter, pidx) pairs, 1-based (schedule.jl order)."""
        memo = self._run_memo
        if memo is not None and memo[0] is steps and memo[1] == steps.shape and memo[2] == steps.dtype:
            n, addr = memo[3], memo[4]  # the same step array again (the driver's repeated window)
        else:
            if (isinstance(steps, np.ndarray) and steps.dtype == np.uint32 and steps.ndim == 2
                    and steps.shape[1] == 2 and steps.flags.c_contiguous):
                arr = steps  # already the emcmc_step[n] layout
                # the memo holds the array itself, so its buffer (and address) stays alive
                self._run_memo = (arr, arr.shape, arr.dtype, arr.shape[0], arr.ctypes.data)
            else:
                arr = np.ascontiguousarray(np.asarray(steps, dtype=np.uint32).reshape(-1, 2))
            n, addr = arr.shape[0], arr.ctypes.data
        if n == 0:
            return
        st = self._lib.emcmc_run(self._h, addr, n)
        if self._cb_error is not None:  # fλ raised on the host while emcmc_run enqueued a readjust
            e, self._cb_error = self._cb_error, None
            raise e
        self._check(st, "emcmc_run")

    def run_iters(self, iter_first: int, n: int, pidx: int = 1):
        it = np.arange(iter_first, iter_first + n, dtype=np.uint32)
        steps = np.stack([it, np.full(n, pidx, dtype=np.uint32)], axis=1)
        self.run(steps)

    def get_proposal_ll(self):
        """sub_ws°.ll of every update (the log-likelihood of its latest proposal), [P][C]."""
        out = np.empty((max(1, self.num_updates), self.cfg.num_chains))
        self._check(self._lib.emcmc_get_proposal_ll(self._h, L.dptr(out)), "emcmc_get_proposal_ll")
        return out

    def synchronize(self, allow_faults=False):
        st = self._lib.emcmc_synchronize(self._h)
        if st == L.CHAIN_FAULT and allow_faults:
            return False
        self._check(st, "emcmc_synchronize")
        return True

    # -- read back ------------------------------------------------------------------
    def get_state(self):
        th = np.empty((self.cfg.num_chains, self.cfg.dim), dtype=np.float64)
        ll = np.empty(self.cfg.num_chains, dtype=np.float64)
        self._check(self._lib.emcmc_get_state(self._h, L.dptr(th), L.dptr(ll)), "emcmc_get_state")
        return th, ll

    def get_chain_stats(self):
        """Rolling acceptance and accepted counts, [P][C] each."""
        P = max(1, self.num_updates)
        ra = np.empty((P, self.cfg.num_chains), dtype=np.float64)
        acc = np.empty((P, self.cfg.num_chains), dtype=np.uint64)
        self._check(
            self._lib.emcmc_get_chain_stats(self._h, L.dptr(ra), acc.ctypes.data_as(C.POINTER(C.c_uint64))),
            "emcmc_get_chain_stats",
        )
        return ra, acc

    def get_update_state(self, pidx: int, nc: int = 0):
        """(ϵ [C][nc] or None, proposed [C], accepted [C]) of update pidx (1-based)."""
        Cn = self.cfg.num_chains
        eps = np.empty((Cn, nc), dtype=np.float64) if nc else None
        pr = np.empty(Cn, dtype=np.uint32)
        ac = np.empty(Cn, dtype=np.uint32)
        self._check(self._lib.emcmc_get_update_state(self._h, pidx, None if eps is None else L.dptr(eps), L.u32ptr(pr),
                                                     L.u32ptr(ac)), "emcmc_get_update_state")
        return eps, pr, ac

    def get_chain_moments(self):
        """GenericChainStats running (mean [C][D], cov [C][D][D]) kept on device."""
        Cn, D = self.cfg.num_chains, self.cfg.dim
        m = np.empty((Cn, D), dtype=np.float64)
        v = np.empty((Cn, D, D), dtype=np.float64)
        self._check(self._lib.emcmc_get_chain_moments(self._h, L.dptr(m), L.dptr(v)), "emcmc_get_chain_moments")
        return m, v

    def get_adaptation_moments(self, pidx: int = 1):
        """HaarioTypeAdaptation (mean [C][n], cov [C][n][n]) of update pidx."""
        Cn, n = self.cfg.num_chains, self._update_n[pidx - 1]
        m = np.empty((Cn, n), dtype=np.float64)
        v = np.empty((Cn, n, n), dtype=np.float64)
        self._check(self._lib.emcmc_get_adaptation_moments(self._h, pidx, L.dptr(m), L.dptr(v)),
                    "emcmc_get_adaptation_moments")
        return m, v

    def get_mix_state(self, pidx: int = 1):
        """(lower Cholesky factor of each chain's Σ_B [C][n][n], Haario M)."""
        Cn, D = self.cfg.num_chains, self._update_n[pidx - 1]
        Lb = np.empty((Cn, D, D), dtype=np.float64)
        M = C.c_uint32()
        self._check(self._lib.emcmc_get_mix_state(self._h, pidx, L.dptr(Lb), C.byref(M)), "emcmc_get_mix_state")
        return Lb, int(M.value)

    def set_mix_lambda_fn(self, pidx: int, f):
        """HaarioTypeAdaptation's fλ(λ, N, mcmc_iter) (adaptation.jl:425), called on the
        host at each readjust; None restores the identity."""
        def tramp(lam, N, it, ctx):  # an exception cannot cross the C ABI: keep it for run() to raise
            try:
                return float(f(lam, int(N), int(it)))
            except BaseException as e:  # noqa: BLE001
                self._cb_error = e
                return lam

        cb = L.LAMBDA_FN(tramp) if f is not None else L.LAMBDA_FN()
        self._flam = cb  # keep the trampoline alive while the handle may call it
        self._check(self._lib.emcmc_set_mix_lambda_fn(self._h, pidx, cb, None), "emcmc_set_mix_lambda_fn")

    def get_mix_lambda(self, pidx: int = 1) -> float:
        v = C.c_double()
        self._check(self._lib.emcmc_get_mix_lambda(self._h, pidx, C.byref(v)), "emcmc_get_mix_lambda")
        return float(v.value)

    def get_faults(self):
        f = np.empty(self.cfg.num_chains, dtype=np.uint32)
        self._check(self._lib.emcmc_get_faults(self._h, L.u32ptr(f)), "emcmc_get_faults")
        return f

    def get_history(self, which: int, iter_first: int, num_iters: int):
        """Returns the raw window; shapes: STATE/PROPOSAL [n][P][C][D], LL [n][P][C],
        ACCEPT [n][P][C] bool (unpacked from the bit rows)."""
        P, Cn, D = self.num_updates, self.cfg.num_chains, self.cfg.dim
        if which in (L.H_STATE, L.H_PROPOSAL):
            out = np.empty((num_iters, P, Cn, D), dtype=np.float64)
        elif which == L.H_LL:
            out = np.empty((num_iters, P, Cn), dtype=np.float64)
        elif which == L.H_ACCEPT:
            words = (Cn + 63) // 64
            out = np.empty((num_iters, P, words), dtype=np.uint64)
        else:
            raise ValueError(which)
        self._check(
            self._lib.emcmc_get_history(self._h, which, iter_first, num_iters, out.ctypes.data, out.nbytes),
            "emcmc_get_history",
        )
        if which == L.H_ACCEPT:
            bits = np.unpackbits(out.view(np.uint8), axis=-1, bitorder="little")
            return bits[..., :Cn].astype(bool)
        return out

    def get_history_bits(self, iter_first: int, num_iters: int):
        """The accept history as stored: [n][P][⌈C/64⌉] u64 words, chain c = bit c % 64 of
        word c // 64 (8× smaller than get_history's unpacked bools, for whole-run checks)."""
        P, Cn = self.num_updates, self.cfg.num_chains
        out = np.empty((num_iters, P, (Cn + 63) // 64), dtype=np.uint64)
        self._check(self._lib.emcmc_get_history(self._h, L.H_ACCEPT, iter_first, num_iters, out.ctypes.data,
                                                out.nbytes), "emcmc_get_history")
        return out

    def get_history_chains(self, which: int, iter_first: int, num_iters: int, chain_first: int, num_chains: int):
        """History window for a chain range: STATE/PROPOSAL [n][P][c][D], LL [n][P][c]."""
        P, D = self.num_updates, self.cfg.dim
        if which in (L.H_STATE, L.H_PROPOSAL):
            out = np.empty((num_iters, P, num_chains, D), dtype=np.float64)
        elif which == L.H_LL:
            out = np.empty((num_iters, P, num_chains), dtype=np.float64)
        else:
            raise ValueError("accept bits: use get_history")
        self._check(
            self._lib.emcmc_get_history_chains(self._h, which, iter_first, num_iters, chain_first, num_chains,
                                               out.ctypes.data, out.nbytes),
            "emcmc_get_history_chains",
        )
        return out

    def stream_history(self, which: int, iter_first: int, num_iters: int, thin: int = 1, out=None):
        """Enqueue an asynchronous copy of iterations iter_first, iter_first+thin, …
        of a history into pinned host memory (emcmc_stream_history).  Returns the
        array (STATE/PROPOSAL [n][P][C][D], LL [n][P][C], ACCEPT [n][P][⌈C/64⌉]
        u64 words); read it after stream_wait()."""
        P, Cn, D = self.num_updates, self.cfg.num_chains, self.cfg.dim
        if which in (L.H_STATE, L.H_PROPOSAL):
            shape, dt = (num_iters, P, Cn, D), np.float64
        elif which == L.H_LL:
            shape, dt = (num_iters, P, Cn), np.float64
        elif which == L.H_ACCEPT:
            shape, dt = (num_iters, P, (Cn + 63) // 64), np.uint64
        else:
            raise ValueError(which)
        if out is None:
            out = PinnedArray(shape, dt)
        assert out.shape == shape and out.dtype == dt and out.flags.c_contiguous
        self._check(self._lib.emcmc_stream_history(self._h, which, iter_first, num_iters, thin, out.ctypes.data,
                                                   out.nbytes), "emcmc_stream_history")
        return out

    def stream_wait(self):
        self._check(self._lib.emcmc_stream_wait(self._h), "emcmc_stream_wait")

    def moments_window(self, iter_first: int, num_iters: int, split: bool = True):
        out = np.empty(3 * self.cfg.dim, dtype=np.float64)
        info = L.EmcmcMoments()
        self._check(
            self._lib.emcmc_moments_window(self._h, iter_first, num_iters, int(split), L.dptr(out), C.byref(info)),
            "emcmc_moments_window",
        )
        D = self.cfg.dim
        return {
            "mean": out[:D].copy(),
            "m2": out[D : 2 * D].copy(),
            "sum_var": out[2 * D :].copy(),
            "num_chains": int(info.num_chains),
            "num_draws": int(info.num_draws),
            "accepted": int(info.accepted),
            "proposed": int(info.proposed),
        }

    def diagnostics(self, iter_first: int, num_iters: int, split: bool = True, comm=None) -> dict:
        """emcmc_diagnostics: this handle's moments over the window, all-gathered over comm
        (an extensible_mcmc.diagnostics.Comm: RCCL or a host all-gather; None = this handle
        alone), merged and turned into split-R̂ by the library.  Collective over comm."""
        from .diagnostics import _diag_dict, _diag_out

        d, arrs = _diag_out(self.cfg.dim)
        st = self._lib.emcmc_diagnostics(self._h, comm.handle if comm else None, iter_first, num_iters, int(split),
                                         C.byref(d))
        if comm is not None and comm.callback_error is not None:
            comm.check(st, "emcmc_diagnostics")
        self._check(st, "emcmc_diagnostics")
        return _diag_dict(d, arrs)

    # -- timing ------------------------------------------------------------------------
    def set_timing(self, enable: bool):
        self._check(self._lib.emcmc_set_timing(self._h, int(enable)), "emcmc_set_timing")

    def get_timing(self, reset: bool = False):
        ms = C.c_double()
        n = C.c_uint64()
        b = C.c_double()
        self._check(
            self._lib.emcmc_get_timing(self._h, C.byref(ms), C.byref(n), C.byref(b), int(reset)),
            "emcmc_get_timing",
        )
        return float(ms.value), int(n.value), float(b.value)

    def kernel_name(self) -> str:
        buf = C.create_string_buffer(256)
        self._check(self._lib.emcmc_kernel_name(self._h, buf, 256), "emcmc_kernel_name")
        return buf.value.decode()

    RTC_ORIGIN = {0: "process", 1: "disk", 2: "compiled", 3: "compiled (cache directory not private: not used)"}

    def rtc_info(self):
        """(origin, seconds) of the handle's run-time compiled kernel: "process"
        (this process's cache), "disk" (the code-object cache), "compiled", or "compiled (cache
        directory not private: not used)" when the cache directory's owner or mode refused it."""
        o, s = C.c_uint32(), C.c_double()
        self._check(self._lib.emcmc_rtc_info(self._h, C.byref(o), C.byref(s)), "emcmc_rtc_info")
        return self.RTC_ORIGIN.get(o.value, str(o.value)), float(s.value)
