"""Cross-chain diagnostics (new functionality: the reference is single-chain;
BASELINE cfg 5).  Each shard reduces its chains on device
(``emcmc_moments_window``) to per-dimension (count, m̄, M2, Σvar) of the
(split-)chain means and variances; shards exchange those with one all-gather
(RCCL over xGMI via ``torch.distributed`` "nccl", or gloo on CPU) and every
rank merges them in rank order with Chan's pairwise update, so M2 never forms
Σm² − (Σm)²/m (which cancels at 1M chains).
"""
from __future__ import annotations

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
    """Split-R̂ (Gelman et al., BDA3 §11.4): B = n·M2/(m−1), W = Σvar/m."""
    mch = m["num_chains"]
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

