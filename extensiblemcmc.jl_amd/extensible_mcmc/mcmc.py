"""MCMC container, MI355X backend/workspaces and the ``run!`` entry point.

Mirrors src/mcmc.jl, src/workspaces.jl and src/run.jl of the reference with a
many-chain device backend: ``MI355XBackend <: MCMCBackend`` is the extension
point the reference provides for exactly this (types.jl:110-117,
workspaces.jl:38,280; docs/src/manual/workspaces.md:70-148).  Each chain is an
independent replica of the reference's single-chain ``run!``; chain c uses the
counter-based variate stream keyed by (seed, first_chain_id + c).

The loop itself (update_workspaces! → update! → update_adaptation!) runs on
the GPU; this module only iterates the schedule on the host, batches the
resulting steps between callback events, and exposes the histories.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import Engine, EngineConfig
from .kernels import (MCMCBackend, MCMCUpdate, PostMCMCStep, PreMCMCStep, UnsupportedPlugin, isdecorator)
from .schedule import MCMCSchedule, Step
from .targets import GsnTargetLaw, LogisticRegressionLaw, UserTargetLaw

_HIST = {"full": L.HIST_FULL, "accept_only": L.HIST_ACCEPT_ONLY}
_LL = {"per_obs": L.LL_PER_OBS, "suffstat": L.LL_SUFFSTAT}


@dataclass
class MI355XBackend(MCMCBackend):
    """Many-chain GPU backend.

    num_chains      chains on this shard (one process per GPU)
    seed            master seed of the counter-based stream
    first_chain_id  global id of the first local chain (sharding)
    device          HIP device ordinal
    history         "full" (state/proposal/ll/accept histories, the reference's
                    outputs) or "accept_only"
    ll_mode         "per_obs" (literal gsn_target.jl loop) or "suffstat"
    chain_moments   keep GenericChainStats' running mean/cov on device
                    (chain_statistics.jl:46-49; always on with GaussianRandomWalkMix)
    """

    num_chains: int = 1
    seed: int = 0
    first_chain_id: int = 0
    device: int = 0
    history: str = "full"
    ll_mode: str = "per_obs"
    roll_window: int = 100
    lanes_per_chain: int = 0
    steps_per_launch: int = 0
    chain_moments: bool = False  # GenericChainStats mean/cov on device (single joint GaussianRandomWalk)


class GenericMCMCBackend(MCMCBackend):
    """The reference's CPU backend flag (types.jl:117).  This package has no CPU
    execution path: selecting it raises, by design (no silent CPU fallback)."""


class MI355XGlobalWorkspace:
    """Global workspace over C chains (replaces GenericGlobalWorkspace, workspaces.jl:209-238).

    ``state`` is [C][D]; histories are fetched from HBM on demand with
    ``state_history(iter_first, n)`` etc. (layout [iter][pidx][chain][coord]).
    """

    def __init__(self, engine: Engine, backend: MI355XBackend, num_mcmc_steps: int, updates, data):
        self.engine = engine
        self.backend = backend
        self.M = num_mcmc_steps
        self.updates = updates
        self.data = data

    @property
    def state(self):
        return self.engine.get_state()[0]

    def num_mcmc_steps(self):
        return self.M

    def num_updt(self):
        return len(self.updates)

    def state_history(self, iter_first: int = 1, num_iters: Optional[int] = None):
        n = self.M - iter_first + 1 if num_iters is None else num_iters
        return self.engine.get_history(L.H_STATE, iter_first, n)

    def state_proposal_history(self, iter_first: int = 1, num_iters: Optional[int] = None):
        n = self.M - iter_first + 1 if num_iters is None else num_iters
        return self.engine.get_history(L.H_PROPOSAL, iter_first, n)

    def chain_stats(self):
        """rolling_ar (current value, chain_statistics.jl:61-64) and accept counts."""
        ra, acc = self.engine.get_chain_stats()
        out = {"rolling_ar": ra, "accepted": acc}
        try:  # GenericChainStats mean/cov, when kept on device
            out["mean"], out["cov"] = self.engine.get_chain_moments()
        except L.EMCMCError as e:
            if e.status != L.STATE_ERROR:
                raise
        return out

    def summary(self, init=False):
        """workspaces.jl:244-262 (over chains)."""
        th = self.state
        lines = [f"Number of MCMC iterations: {self.M}", f"Number of chains: {th.shape[0]}",
                 f"Number of updates at each MCMC iteration: {self.num_updt()}"]
        if not init:
            lines.append(f"Cross-chain mean of θ: {th.mean(axis=0)}")
        return "\n".join(lines)


class MI355XLocalWorkspace:
    """Per-update local workspace view (replaces GenericLocalWorkspace, workspaces.jl:453-476)."""

    def __init__(self, gws: MI355XGlobalWorkspace, pidx: int, update):
        self.gws = gws
        self.pidx = pidx
        self.update = update
        self.updt_name = type(update).__name__

    @property
    def ll(self):
        return self.gws.engine.get_state()[1]

    def ll_history(self, iter_first: int = 1, num_iters: Optional[int] = None):
        n = self.gws.M - iter_first + 1 if num_iters is None else num_iters
        return self.gws.engine.get_history(L.H_LL, iter_first, n)[:, self.pidx - 1, :]

    def acceptance_history(self, iter_first: int = 1, num_iters: Optional[int] = None):
        n = self.gws.M - iter_first + 1 if num_iters is None else num_iters
        return self.gws.engine.get_history(L.H_ACCEPT, iter_first, n)[:, self.pidx - 1, :]

    def accepted(self, i: int):
        return self.acceptance_history(i, 1)[0]

    def name_of_update(self):
        return self.updt_name


def strip_decorators(ud):
    """mcmc.jl:56"""
    return [u for u in ud if not isdecorator(u)]


def get_decorators(ud):
    """mcmc.jl:63"""
    return [u for u in ud if isdecorator(u)]


class MCMC:
    """``MCMC(updates_and_decorators; backend)`` (mcmc.jl:32-49)."""

    def __init__(self, updt_and_decor: Sequence, backend: Optional[MCMCBackend] = None):
        self.updates_and_decorators = list(updt_and_decor)
        self.updates: List[MCMCUpdate] = strip_decorators(self.updates_and_decorators)
        self.backend = MI355XBackend() if backend is None else backend
        self.schedule: Optional[MCMCSchedule] = None
        self.workspace: Optional[MI355XGlobalWorkspace] = None


def init_global_workspace(backend: MCMCBackend, num_mcmc_steps: int, updates, data, theta_init, **kwargs):
    """workspaces.jl:38 / :215-234 for the device backend."""
    if not isinstance(backend, MI355XBackend):
        raise UnsupportedPlugin(
            f"backend {type(backend).__name__} has no device implementation; use MI355XBackend")
    P = data["P"]
    if not isinstance(P, (GsnTargetLaw, LogisticRegressionLaw, UserTargetLaw)):
        raise UnsupportedPlugin(f"target law {type(P).__name__} has no device plugin yet")
    th0 = np.asarray(theta_init, dtype=float)
    D = th0.shape[-1]
    C = backend.num_chains
    if th0.ndim == 1:
        th0 = np.broadcast_to(th0, (C, D))
    cfg = EngineConfig(dim=D, num_chains=C, num_mcmc_steps=num_mcmc_steps, seed=backend.seed,
                       first_chain_id=backend.first_chain_id, device=backend.device,
                       history_mode=_HIST[backend.history], roll_window=backend.roll_window,
                       lanes_per_chain=backend.lanes_per_chain, steps_per_launch=backend.steps_per_launch,
                       chain_moments=backend.chain_moments)
    eng = Engine(cfg)
    try:
        for u in updates:
            u.to_device(eng)
        P.to_device(eng, _LL[backend.ll_mode], data["obs"])
    except L.EMCMCError as e:  # the engine's own "no device plugin" verdicts
        if e.status == L.UNSUPPORTED_PLUGIN:
            raise UnsupportedPlugin(str(e)) from e
        raise
    eng.set_state(np.ascontiguousarray(th0))
    return MI355XGlobalWorkspace(eng, backend, num_mcmc_steps, updates, data)


def extra_schedule_params(workspace, updates_and_decorators, **kwargs):
    """mcmc.jl:111-117"""
    return {}


def init(mcmc: MCMC, num_mcmc_steps: int, data, theta_init, exclude_updates=(), **kwargs):
    """``init!`` (mcmc.jl:83-109)."""
    mcmc.workspace = init_global_workspace(mcmc.backend, num_mcmc_steps, mcmc.updates, data, theta_init, **kwargs)
    mcmc.schedule = MCMCSchedule(num_mcmc_steps, len(mcmc.updates), exclude_updates,
                                 **extra_schedule_params(mcmc.workspace, mcmc.updates_and_decorators, **kwargs))


def create_workspaces(backend, mcmc: MCMC):
    """workspaces.jl:362-371"""
    return [MI355XLocalWorkspace(mcmc.workspace, i + 1, u) for i, u in enumerate(mcmc.updates)]


def _run_loop(global_ws, local_wss, updates, schedule, callbacks):
    """``__run!`` (run.jl:64-83): the per-step body executes on the device; the
    host flushes the accumulated steps whenever a callback is about to fire."""
    pending = []

    def flush():
        if pending:
            global_ws.engine.run(pending)
            pending.clear()

    for step in schedule:
        pre = [cb for cb in callbacks if cb.check_if_execute(step, PreMCMCStep())]
        if pre:
            flush()
            global_ws.engine.synchronize()
            for cb in pre:
                cb.execute(global_ws, local_wss, step, PreMCMCStep())
        pending.append((step.mcmciter, step.pidx))
        post = [cb for cb in callbacks if cb.check_if_execute(step, PostMCMCStep())]
        if post:
            flush()
            global_ws.engine.synchronize()
            for cb in post:
                cb.execute(global_ws, local_wss, step, PostMCMCStep())
    flush()
    global_ws.engine.synchronize(allow_faults=True)


def run(mcmc: MCMC, num_mcmc_steps: int, data, theta_init, callbacks=(), **kwargs):
    """``run!(mcmc, num_mcmc_steps, data, θinit, callbacks; kwargs...)`` (run.jl:34-54).

    Returns ``(global_ws, local_wss)``.  ``exclude_updates`` is honoured as in
    the reference (run.jl:43).
    """
    init(mcmc, num_mcmc_steps, data, theta_init, kwargs.get("exclude_updates", ()), **kwargs)
    local_wss = create_workspaces(mcmc.backend, mcmc)
    for cb in callbacks:
        cb.init(mcmc.workspace)
    _run_loop(mcmc.workspace, local_wss, mcmc.updates, mcmc.schedule, list(callbacks))
    for i, u in enumerate(mcmc.updates):  # adapted ϵ / counters, as the reference mutates them
        if hasattr(u, "pull_device_state"):
            u.pull_device_state(mcmc.workspace.engine, i + 1)
    for cb in callbacks:
        cb.cleanup(mcmc.workspace, local_wss, Step(None, None, num_mcmc_steps, 1))
    return mcmc.workspace, local_wss


run_ = run  # closest Python spelling of `run!`
