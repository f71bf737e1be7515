"""Cross-chain diagnostics (new functionality: the reference is single-chain;
BASELINE cfg 5).  Each shard reduces its chains on device
(``emcmc_moments_window``) to 3·D fp64 sums + counts; shards combine with one
all-reduce (RCCL over xGMI via ``torch.distributed`` "nccl", or gloo on CPU).
"""
from __future__ import annotations

import numpy as np


def pack(m: dict) -> np.ndarray:
    return np.concatenate([
        m["sum_mean"], m["sum_mean_sq"], m["sum_var"],
        np.array([m["num_chains"], m["accepted"], m["proposed"]], dtype=np.float64),
    ])


def unpack(v: np.ndarray, D: int, num_draws: int) -> dict:
    return {
        "sum_mean": v[:D], "sum_mean_sq": v[D:2 * D], "sum_var": v[2 * D:3 * D],
        "num_chains": int(round(v[3 * D])), "accepted": int(round(v[3 * D + 1])),
        "proposed": int(round(v[3 * D + 2])), "num_draws": num_draws,
    }


def rhat_from_sums(m: dict) -> dict:
    """Split-R̂ (Gelman et al., BDA3 §11.4) from per-(half-)chain sums."""
    mch = m["num_chains"]
    n = m["num_draws"]
    S1, S2, S3 = (np.asarray(m[k], dtype=np.float64) for k in ("sum_mean", "sum_mean_sq", "sum_var"))
    mean = S1 / mch
    B = n / (mch - 1) * (S2 - S1 * S1 / mch)
    W = S3 / mch
    var_plus = (n - 1) / n * W + B / n
    rhat = np.sqrt(var_plus / W)
    acc = m["accepted"] / max(1, m["proposed"])
    return {"rhat": rhat, "mean": mean, "W": W, "B": B, "accept_rate": acc}


def allreduce_sums(m: dict, D: int, group=None, device=None) -> dict:
    """Sum the shard's diagnostics over all ranks (one all-reduce of 3·D+3 doubles)."""
    import torch
    import torch.distributed as dist

    v = pack(m)
    if not (dist.is_available() and dist.is_initialized()):
        return m
    t = torch.from_numpy(v.copy())
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return unpack(t.cpu().numpy(), D, m["num_draws"])
