"""The reference-shaped API end to end on the GPU: MCMC(...) + run(...) with the
MI355X backend, mirroring the reference's "mcmc" testset and tutorial
(test/runtests.jl:87-114, docs/src/tutorials/mean_of_bivariate_gaussian.md)."""
import numpy as np
import pytest

from extensible_mcmc import (MCMC, GaussianRandomWalk, GsnTargetLaw, ImproperPrior, MI355XBackend,
                             RandomWalkUpdate, REPLCallback, SavingCallback, UniformRandomWalk,
                             UnsupportedPlugin, run)
from extensible_mcmc import workloads as W

from helpers import run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(require_gpu):
    pass


def test_run_bivariate_joint_gaussian_rw(oracle, tmp_path):
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(GaussianRandomWalk(0.5 * np.eye(2)), [1, 2], prior=ImproperPrior())],
                backend=MI355XBackend(num_chains=256, seed=w.seed))
    lines = []
    saver = SavingCallback(path=str(tmp_path), chains=(0, 5))
    ws, lwss = run(mcmc, 1000, dict(P=GsnTargetLaw([1.0, 2.0], [[1.0, 0.5], [0.5, 1.0]]), obs=w.obs),
                   [0.0, 0.0], [saver, REPLCallback(print_every_k_iter=250, printer=lines.append)])
    o = run_oracle(oracle, w, 256, 1000)
    assert np.array_equal(ws.state, o["state"].theta)
    assert np.array_equal(lwss[0].acceptance_history(1, 1000), o["acc"])
    assert np.array_equal(ws.state_history(1, 1000)[:, 0], o["theta"])
    # SavingCallback: rows for iterations 1..M-1 (callbacks.jl:223), reference row format
    rows = (tmp_path / "mcmc_results_chain0.csv").read_text().splitlines()
    assert len(rows) == 999
    assert rows[0].startswith("1, 1, !, ") and rows[0].count("!") == 5
    vals = rows[10].split(", ")
    assert float(vals[3]) == o["theta"][10, 0, 0]
    assert any("1000.1" in l for l in lines) and any("successful" in l for l in lines)


def test_unsupported_plugins_raise_not_fallback():
    w = W.ref_test()
    mcmc = MCMC([RandomWalkUpdate(UniformRandomWalk([1.0]), [1]), RandomWalkUpdate(UniformRandomWalk([1.0]), [2])],
                backend=MI355XBackend(num_chains=8))
    with pytest.raises(UnsupportedPlugin):
        run(mcmc, 10, dict(P=GsnTargetLaw([1.0, 2.0]), obs=w.obs), [0.0, 0.0])
