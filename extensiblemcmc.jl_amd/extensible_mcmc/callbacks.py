"""Callbacks (reference src/callbacks.jl): host-side I/O around the device loop.

With many chains, ``SavingCallback`` writes the reference's CSV row format
(callbacks.jl:246-256) for a chosen subset of chains (default: chain 0), one
file per chain.  ``REPLCallback`` prints progress for chain 0
(callbacks.jl:306-319).
"""
from __future__ import annotations

import datetime as _dt
import os
from typing import Sequence

import numpy as np

from .kernels import PostMCMCStep, PreMCMCStep


class Callback:
    def init(self, ws):  # callbacks.jl:27
        pass

    def check_if_execute(self, step, flag) -> bool:  # callbacks.jl:55
        return False

    def execute(self, global_ws, local_wss, step, flag):  # callbacks.jl:70
        pass

    def cleanup(self, ws, local_wss, step):  # callbacks.jl:85 (arity as called at run.jl:51)
        pass


def find_available_name(path, filename, disambig_num="", extension=".csv"):
    """callbacks.jl:173-180"""
    while True:
        proposal = os.path.join(path, f"{filename}{disambig_num}{extension}")
        if not os.path.isfile(proposal):
            return proposal
        disambig_num = "1" if disambig_num == "" else str(int(disambig_num) + 1)


def julia_float_string(x: float) -> str:
    """Julia's ``string(::Float64)`` (Base.Ryu.writeshortest as ``show`` calls it):
    the shortest round-trip digits d₁…dₙ (Python's repr yields the same digit
    string) of x = 0.d₁…dₙ × 10^pt, printed in plain decimal when −4 ≤ pt − 1 ≤ 5
    (1.0e-5, 0.0001, 100000.0, 1.0e6) and as d₁.d₂…dₙe±k otherwise; integral
    values keep a trailing ".0", a single digit gets ".0" in scientific form
    ("1.0e-5"), and the exponent has no "+" or padding.  NaN, Inf, -Inf as Julia."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Inf" if x > 0 else "-Inf"
    if x == 0.0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))
    if "e" in r:
        m, e = r.split("e")
        e = int(e)
    else:
        m, e = r, 0
    ip, _, fp = m.partition(".")
    digits = (ip + fp).lstrip("0")
    # position of the decimal point relative to the first significant digit
    pt = len(ip.lstrip("0")) + e if ip.lstrip("0") else e - (len(fp) - len(fp.lstrip("0")))
    digits = digits.rstrip("0") or "0"
    n = len(digits)
    k = pt - 1  # scientific exponent
    if -4 <= k <= 5:
        if pt <= 0:
            body = "0." + "0" * (-pt) + digits
        elif pt < n:
            body = digits[:pt] + "." + digits[pt:]
        else:
            body = digits + "0" * (pt - n) + ".0"
    else:
        body = digits[0] + "." + (digits[1:] if n > 1 else "0") + f"e{k}"
    return sign + body


def _fmt(x) -> str:
    """One CSV entry as Julia's string interpolation writes it (callbacks.jl:249-253)."""
    if isinstance(x, (bool, np.bool_)):
        return "true" if x else "false"
    return julia_float_string(float(x))


class SavingCallback(Callback):
    """``SavingCallback(; save_at_the_end=true, save_at_iters=[], overwrite_at_save=false,
    filename="mcmc_results", add_datestamp=false, path=".")`` (callbacks.jl:125-164)."""

    def __init__(self, save_at_the_end=True, save_at_iters=(), overwrite_at_save=False, filename="mcmc_results",
                 add_datestamp=False, path=".", chains: Sequence[int] = (0,)):
        stamp = "_" + _dt.datetime.now().strftime("%Y-%m-%d_%H:%M:%S") if add_datestamp else ""
        filename = f"{filename}{stamp}"
        self.chains = list(chains)
        self.filenames = {}
        for c in self.chains:
            stem = filename if len(self.chains) == 1 else f"{filename}_chain{c}"
            self.filenames[c] = (os.path.join(path, stem + ".csv") if overwrite_at_save
                                 else find_available_name(path, stem, ""))
        self.save_at_the_end = save_at_the_end
        self.save_intermediate = len(save_at_iters) > 0
        self.save_at_iters = sorted(int(i) for i in save_at_iters)

    @property
    def filename(self):
        return self.filenames[self.chains[0]]

    def init(self, ws):
        for fn in self.filenames.values():
            open(fn, "w").close()

    def check_if_execute(self, step, flag):
        if not isinstance(flag, PreMCMCStep) or not self.save_intermediate:
            return False
        return step.mcmciter in self.save_at_iters and step.pidx == 1

    def cleanup(self, ws, local_wss, step):
        if self.save_at_the_end:
            self.execute(ws, local_wss, step, None)

    def _start(self, step):
        if not self.save_intermediate:
            return 1
        import bisect
        i = bisect.bisect_left(self.save_at_iters, step.mcmciter)
        return 1 if i == 0 else self.save_at_iters[i - 1]

    def execute(self, ws, local_wss, step, flag):
        first = self._start(step)
        last = step.mcmciter - 1  # callbacks.jl:223
        if last < first:
            return
        n = last - first + 1
        th = ws.state_history(first, n)
        thp = ws.state_proposal_history(first, n)
        ll = np.stack([lw.ll_history(first, n) for lw in local_wss], axis=1)
        acc = np.stack([lw.acceptance_history(first, n) for lw in local_wss], axis=1)
        P = len(local_wss)
        for c, fn in self.filenames.items():
            with open(fn, "a") as f:
                for k in range(n):
                    i = first + k
                    for j in range(P):
                        row = [f"{i}, {j + 1}, ", "!, "]
                        row += [f"{_fmt(v)}, " for v in th[k, j, c]]
                        row.append("!, ")
                        row += [f"{_fmt(v)}, " for v in thp[k, j, c]]
                        row.append("!, ")
                        row.append(f"{_fmt(ll[k, j, c])}, ")
                        row.append("!, ")
                        # ll° history is never written by the reference (workspaces.jl:337
                        # ignores i; run.jl:258,332 self-assign): its zero-initialised value
                        row.append(f"{_fmt(0.0)}, ")
                        row.append("!,")
                        row.append(f"{_fmt(bool(acc[k, j, c]))}, ")
                        f.write("".join(row) + "\n")


class REPLCallback(Callback):
    """``REPLCallback(; print_every_k_iter=100, show_all_upates=true, basic_info_only=true)``
    (callbacks.jl:279-291); reports chain 0 and the cross-chain acceptance."""

    def __init__(self, print_every_k_iter=100, show_all_upates=True, basic_info_only=True, printer=print):
        self.print_every_k_iter = print_every_k_iter
        self.show_all_updates = show_all_upates
        self.basic_info_only = basic_info_only
        self.printer = printer

    def init(self, ws):
        self.printer("*" * 40)
        self.printer("Initializing an MCMC chain")
        self.printer(ws.summary(init=True))
        self.printer("* * *")

    def check_if_execute(self, step, flag):
        if not isinstance(flag, PostMCMCStep):
            return False
        if step.mcmciter % self.print_every_k_iter != 0:
            return False
        return self.show_all_updates or step.pidx == 1

    def execute(self, ws, local_wss, step, flag):
        lw = local_wss[step.pidx - 1]
        M = step.mcmciter
        ll = lw.ll_history(M, 1)[0]
        acc = lw.acceptance_history(M, 1)[0]
        self.printer("- - - - - - - - - - -")
        self.printer(f"{M}.{step.pidx} {lw.name_of_update()}")
        self.printer(f"\tchain 0 ll: {ll[0]:.4g}, a/r: {'✔' if acc[0] else '✗'}; "
                     f"accepted at this step: {acc.mean():.3f} of {acc.size} chains")
        if not self.basic_info_only:
            self.printer(f"\t\tθ : {np.round(ws.state[0], 4)}")

    def cleanup(self, ws, local_wss, step):
        self.printer("\n\nMCMC sampling has been successful!")
        self.printer("Doing some clean-up and finishing...")
        self.printer("\n⋆ ⋆ ⋆\n")
