"""A do-nothing stand-in for extensible_mcmc.engine.Engine, loaded by bench.py only
when EMCMC_BENCH_STUB_ENGINE=1 (test infrastructure: never a measured path; the
line it produces says "stub_engine": true).  It lets a CPU test drive
`bench.py --gpus N` end to end (launcher, gloo ranks, timing windows, the
diagnostics all-gather) without a GPU.  The moments it reports depend on the
shard's global chain ids, so the all-gather's merge is not trivial."""
import numpy as np


class EngineConfig:
    def __init__(self, dim, num_chains, num_mcmc_steps, seed=0, first_chain_id=0, **kw):
        self.dim, self.num_chains, self.num_mcmc_steps = dim, num_chains, num_mcmc_steps
        self.seed, self.first_chain_id = seed, first_chain_id
        self.kw = kw


class Engine:
    def __init__(self, cfg: EngineConfig):
        self.cfg = cfg
        self.timing = False
        self.launches = 0
        self.steps_run = 0

    def __getattr__(self, name):  # add_*_update, set_*_target: accepted and ignored
        if name.startswith(("add_", "set_")):
            return lambda *a, **k: None
        raise AttributeError(name)

    def run_iters(self, it, n, pidx=1):
        self.steps_run += n

    def run(self, steps):
        self.steps_run += len(steps)
        if self.timing:
            self.launches += max(1, len(steps) // 100)

    def synchronize(self, allow_faults=False):
        pass

    def set_timing(self, enable):
        self.timing = bool(enable)

    def get_timing(self, reset=False):
        n = self.launches
        if reset:
            self.launches = 0
        n = max(n, 1)
        return 0.1 * n, n, 1.0e6 * n

    def moments_window(self, iter_first, num_iters, split=True):
        D, C = self.cfg.dim, self.cfg.num_chains
        halves = 2 if split else 1
        ids = self.cfg.first_chain_id + np.arange(C * halves, dtype=np.float64)
        means = np.sin(ids[:, None] * 1e-3 + np.arange(D)[None, :])
        return {"mean": means.mean(0), "m2": ((means - means.mean(0)) ** 2).sum(0),
                "sum_var": np.full(D, 1.5 * C * halves), "num_chains": C * halves,
                "num_draws": num_iters // halves, "accepted": C * num_iters // 4, "proposed": C * num_iters}

    def diagnostics(self, iter_first, num_iters, split=True, comm=None):
        from extensible_mcmc import diagnostics as DG  # the library's merge (emcmc_diagnostics_merge)

        m = self.moments_window(iter_first, num_iters, split)
        return DG.merge_c(DG.pack(m), self.cfg.dim, m["num_draws"], comm)

    def get_faults(self):
        return np.zeros(self.cfg.num_chains, dtype=np.uint32)

    def kernel_name(self):
        return "stub"

    def close(self):
        pass
