"""Cross-chain diagnostics (new functionality: the reference is single-chain;
BASELINE cfg 5).  Each shard reduces its chains on device
(``emcmc_moments_window``) to per-dimension (count, m̄, M2, Σvar) of the
(split-)chain means and variances; shards exchange those with one all-gather
(RCCL over xGMI via ``torch.distributed`` "nccl", or gloo on CPU) and every
rank merges them in rank order with Chan's pairwise update, so M2 never forms
Σm² − (Σm)²/m (which cancels at 1M chains).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def pack(m: dict) -> np.ndarray:
    return np.concatenate([
        np.array([m["num_chains"]], dtype=np.float64), m["mean"], m["m2"], m["sum_var"],
        np.array([m["accepted"], m["proposed"]], dtype=np.float64),
    ])


def unpack(v: np.ndarray, D: int, num_draws: int) -> dict:
    return {
        "num_chains": int(round(v[0])), "mean": v[1:1 + D].copy(), "m2": v[1 + D:1 + 2 * D].copy(),
        "sum_var": v[1 + 2 * D:1 + 3 * D].copy(), "accepted": int(round(v[1 + 3 * D])),
        "proposed": int(round(v[2 + 3 * D])), "num_draws": num_draws,
    }


def from_chain_moments(means: np.ndarray, vars_: np.ndarray, num_draws: int, accepted=0, proposed=0) -> dict:
    """Moments of one shard from its per-(half-)chain means/variances [m][D] (host restatement)."""
    return {"num_chains": int(means.shape[0]), "mean": means.mean(0),
            "m2": ((means - means.mean(0)) ** 2).sum(0), "sum_var": vars_.sum(0),
            "num_draws": num_draws, "accepted": int(accepted), "proposed": int(proposed)}


def merge(parts: list[dict]) -> dict:
    """Chan et al.'s pairwise combination of shard moments, left to right (rank order)."""
    out = dict(parts[0])
    out["mean"] = np.array(out["mean"], dtype=np.float64)
    out["m2"] = np.array(out["m2"], dtype=np.float64)
    out["sum_var"] = np.array(out["sum_var"], dtype=np.float64)
    for b in parts[1:]:
        na, nb = float(out["num_chains"]), float(b["num_chains"])
        if nb == 0:
            continue
        n = na + nb
        dl = np.asarray(b["mean"]) - out["mean"]
        out["mean"] = out["mean"] + dl * (nb / n)
        out["m2"] = (out["m2"] + np.asarray(b["m2"])) + dl * dl * (na * nb / n)
        out["sum_var"] = out["sum_var"] + np.asarray(b["sum_var"])
        out["num_chains"] = int(n)
        out["accepted"] += int(b["accepted"])
        out["proposed"] += int(b["proposed"])
    return out


def rhat_from_moments(m: dict) -> dict:
    """Split-R̂ (Gelman et al., BDA3 §11.4): B = n·M2/(m−1), W = Σvar/m.  Fewer than two
    (half-)chains: ValueError (the library's emcmc_diagnostics_merge returns INVALID_ARG)."""
    mch = m["num_chains"]
    if mch < 2:
        raise ValueError(f"split-R̂ needs at least 2 (half-)chains over all ranks, got {mch}")
    n = m["num_draws"]
    mean = np.asarray(m["mean"], dtype=np.float64)
    B = n / (mch - 1) * np.asarray(m["m2"], dtype=np.float64)
    W = np.asarray(m["sum_var"], dtype=np.float64) / mch
    var_plus = (n - 1) / n * W + B / n
    rhat = np.sqrt(var_plus / W)
    acc = m["accepted"] / max(1, m["proposed"])
    return {"rhat": rhat, "mean": mean, "W": W, "B": B, "accept_rate": acc}


def allgather_moments(m: dict, D: int, group=None, device=None) -> dict:
    """All-gather every rank's shard moments (3·D+3 doubles each) and merge them
    in rank order; every rank ends with the same global moments."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return m
    v = torch.from_numpy(pack(m))
    if device is not None:
        v = v.to(device)
    world = dist.get_world_size(group)
    out = torch.empty(world * v.numel(), dtype=v.dtype, device=v.device)
    dist.all_gather_into_tensor(out, v, group=group)
    rows = out.cpu().numpy().reshape(world, -1)
    return merge([unpack(r, D, m["num_draws"]) for r in rows])


# ---- the same through the C ABI (include/emcmc.h: emcmc_comm_*, emcmc_diagnostics) ----------
# The library all-gathers the records itself (RCCL over xGMI, or a host all-gather the
# caller supplies) and merges them in C with the arithmetic above, bit for bit; this is
# the path the Julia shim and bench.py use.

def _diag_out(D: int):
    from . import _lib as L

    arrs = {k: np.empty(D) for k in ("mean", "m2", "sum_var", "W", "B", "rhat")}
    d = L.EmcmcDiag()
    for k, a in arrs.items():
        setattr(d, k, L.dptr(a))
    return d, arrs


def _diag_dict(d, arrs) -> dict:
    return {**arrs, "num_chains": int(d.num_chains), "num_draws": int(d.num_draws), "accepted": int(d.accepted),
            "proposed": int(d.proposed), "accept_rate": float(d.accept_rate), "max_rhat": float(d.max_rhat),
            "nranks": int(d.nranks)}


class Comm:
    """An emcmc_comm: the ranks of one job for emcmc_diagnostics.  `rccl` joins one GPU per
    rank through RCCL (rank 0 draws the unique id, the caller broadcasts it); `host` wraps
    the caller's own all-gather of float64 vectors (gloo, MPI)."""

    def __init__(self, handle, nranks: int, rank: int, keep=None):
        self._h, self.nranks, self.rank, self._keep = handle, nranks, rank, keep
        self.callback_error = None

    @staticmethod
    def unique_id() -> bytes:
        from . import _lib as L

        buf = (C.c_uint8 * L.COMM_ID_BYTES)()
        st = L.lib().emcmc_comm_unique_id(buf)
        if st != L.OK:
            raise L.EMCMCError(st, "emcmc_comm_unique_id", L.lib().emcmc_comm_last_error(None).decode())
        return bytes(buf)

    @classmethod
    def rccl(cls, nranks: int, rank: int, device: int, uid: bytes) -> "Comm":
        from . import _lib as L

        h = C.c_void_p()
        idb = (C.c_uint8 * L.COMM_ID_BYTES).from_buffer_copy(uid)
        st = L.lib().emcmc_comm_init(C.byref(h), nranks, rank, device, idb)
        if st != L.OK:
            raise L.EMCMCError(st, "emcmc_comm_init", L.lib().emcmc_comm_last_error(None).decode())
        return cls(h, nranks, rank)

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "Comm":
        """An RCCL comm over the ranks of a torch.distributed group: rank 0's unique id
        travels with broadcast_object_list (any backend)."""
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls.rccl(world, rank, device, obj[0])

    @classmethod
    def host(cls, nranks: int, rank: int, allgather) -> "Comm":
        """allgather(send: ndarray[count]) -> ndarray[nranks·count] in rank order."""
        from . import _lib as L

        def tramp(send, recv, count, ctx):
            try:
                s = np.ctypeslib.as_array(send, shape=(count,)).copy()
                r = np.asarray(allgather(s), dtype=np.float64).reshape(-1)
                if r.size != nranks * count:
                    raise ValueError(f"all-gather returned {r.size} doubles, expected {nranks * count}")
                np.ctypeslib.as_array(recv, shape=(nranks * count,))[:] = r
                return 0
            except BaseException as e:  # an exception cannot cross the C ABI
                comm.callback_error = e
                return 1

        fn = L.ALLGATHER_FN(tramp)
        h = C.c_void_p()
        st = L.lib().emcmc_comm_init_host(C.byref(h), nranks, rank, fn, None)
        if st != L.OK:
            raise L.EMCMCError(st, "emcmc_comm_init_host")
        comm = cls(h, nranks, rank, keep=fn)
        return comm

    @classmethod
    def torch_host(cls, group=None, device=None) -> "Comm":
        """A host comm over a torch.distributed group: CPU tensors (gloo), or tensors on
        `device` (a torch device, e.g. under the nccl backend)."""
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(group)

        def ag(send):
            t = torch.from_numpy(send)
            if device is not None:
                t = t.to(device)
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t, group=group)
            return out.cpu().numpy()

        return cls.host(world, dist.get_rank(group), ag)

    @property
    def handle(self):
        return self._h

    def check(self, st: int, where: str):
        from . import _lib as L

        if self.callback_error is not None:
            e, self.callback_error = self.callback_error, None
            raise e
        if st != L.OK:
            msg = L.lib().emcmc_comm_last_error(self._h)
            raise L.EMCMCError(st, where, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "_h", None):
            from . import _lib as L

            L.lib().emcmc_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def merge_c(record: np.ndarray, D: int, num_draws: int, comm: Comm | None = None) -> dict:
    """emcmc_diagnostics_merge: this rank's record (pack() layout) all-gathered over comm
    (None: this rank alone), merged and turned into split-R̂ by the library."""
    from . import _lib as L

    rec = np.ascontiguousarray(record, dtype=np.float64)
    assert rec.size == 3 * D + 3
    d, arrs = _diag_out(D)
    st = L.lib().emcmc_diagnostics_merge(comm.handle if comm else None, L.dptr(rec), D, num_draws, C.byref(d))
    if comm is not None:
        comm.check(st, "emcmc_diagnostics_merge")
    elif st != L.OK:
        raise L.EMCMCError(st, "emcmc_diagnostics_merge", L.lib().emcmc_comm_last_error(None).decode())
    return _diag_dict(d, arrs)
