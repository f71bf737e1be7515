"""MCMCSchedule — host-side driver of the hot loop (reference src/schedule.jl).

The schedule stays on the host: every chain follows the same (mcmciter, pidx)
sequence, so the device receives the resulting step list (include/emcmc.h
``emcmc_step``).  Semantics follow the reference exactly, including:
  * the start state is yielded without an exclusion check (schedule.jl:56-66);
  * ``transition`` skips excluded (iter, pidx) recursively (schedule.jl:77-89);
  * ``reschedule!`` may be called mid-iteration and is seen by the very next
    ``transition`` (schedule.jl:105-118).
Indices are 1-based, as in the reference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, NamedTuple, Optional


class JRange:
    """Julia's inclusive range ``start:stop`` / ``start:step:stop`` (an OrdinalRange)."""

    __slots__ = ("start", "stop", "step")

    def __init__(self, start: int, stop: int, step: int = 1):
        if step == 0:
            raise ValueError("step cannot be zero")
        self.start, self.stop, self.step = int(start), int(stop), int(step)

    def __contains__(self, x: int) -> bool:
        if self.step > 0:
            if x < self.start or x > self.stop:
                return False
        else:
            if x > self.start or x < self.stop:
                return False
        return (x - self.start) % self.step == 0

    def __iter__(self):
        return iter(range(self.start, self.stop + (1 if self.step > 0 else -1), self.step))

    def __repr__(self):
        return f"{self.start}:{self.stop}" if self.step == 1 else f"{self.start}:{self.step}:{self.stop}"

    def __eq__(self, o):
        return isinstance(o, JRange) and list(self) == list(o)


def _as_range(r) -> JRange:
    if isinstance(r, JRange):
        return r
    if isinstance(r, range):
        if len(r) == 0:
            return JRange(0, -1)
        return JRange(r.start, r[-1], r.step)
    if isinstance(r, int):
        return JRange(r, r)
    raise TypeError(f"cannot interpret {r!r} as a range of MCMC iterations")


def _as_indices(x) -> Iterable[int]:
    if isinstance(x, int):
        return [x]
    return list(_as_range(x)) if isinstance(x, (JRange, range)) else list(x)


class Step(NamedTuple):
    prev_mcmciter: Optional[int]
    prev_pidx: Optional[int]
    mcmciter: int
    pidx: int


class _ExcludeDict(dict):
    """DefaultDict{Int64, OrdinalRange}(0:0) (schedule.jl:32)."""

    def __missing__(self, key):
        return JRange(0, 0)


@dataclass
class MCMCSchedule:
    """``MCMCSchedule(num_mcmc_steps, num_updates, exclude_updates=[]; start, backend, extra_info)``
    (schedule.jl:17-46).  ``exclude_updates`` is a list of ``(update_indices, iteration_range)``."""

    num_mcmc_steps: int
    num_updates: int
    exclude_updates: object = ()
    start: Optional[Step] = None
    backend: object = None
    extra_info: object = None

    def __post_init__(self):
        excl = _ExcludeDict()
        for idxs, rng in self.exclude_updates:
            for idx in _as_indices(idxs):
                excl[int(idx)] = _as_range(rng)
        self.exclude_updates = excl
        if self.start is None:
            self.start = Step(None, None, 1, 1)

    # schedule.jl:56-66
    def __iter__(self):
        state = self.start
        while True:
            if state.mcmciter > self.num_mcmc_steps:
                return
            tmp = Step(state.mcmciter, state.pidx, state.mcmciter, state.pidx)
            new_state = self.transition(tmp)
            yield state
            state = new_state

    # schedule.jl:77-89 (recursion unrolled into a loop)
    def transition(self, state: Step) -> Step:
        while True:
            reset = state.pidx == self.num_updates
            new_state = Step(
                state.prev_mcmciter,
                state.prev_pidx,
                state.mcmciter + (1 if reset else 0),
                1 if reset else state.pidx + 1,
            )
            if new_state.mcmciter in self.exclude_updates[new_state.pidx]:
                state = new_state
                continue
            return new_state

    def steps(self):
        """The (mcmciter, pidx) sequence of a full iteration (host → device step list)."""
        return [(s.mcmciter, s.pidx) for s in self]


def reschedule(schedule: MCMCSchedule, num_new_updates: int = 0, idxes_to_remove=(), idxes_to_add=()):
    """``reschedule!`` (schedule.jl:105-118)."""
    schedule.num_updates += num_new_updates
    for idx in idxes_to_remove:
        schedule.exclude_updates[int(idx)] = JRange(1, schedule.num_mcmc_steps)
    for idx, rng in idxes_to_add:
        schedule.exclude_updates[int(idx)] = _as_range(rng)


reschedule_ = reschedule  # spelling close to the reference's `reschedule!`
