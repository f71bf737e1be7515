"""Host-side bookkeeping of the Engine wrapper, checked without a GPU: the
ctypes call into emcmc_add_update is replaced by a recorder, so only the Python
packing and the per-update shape list are exercised."""
import ctypes as C

import numpy as np

from extensible_mcmc import _lib as L
from extensible_mcmc.engine import Engine, EngineConfig


class _RecordingLib:
    """Stands in for libemcmc.so: emcmc_add_update records the descriptor."""

    def __init__(self):
        self.added = []

    def emcmc_add_update(self, h, pu):
        u = C.cast(pu, C.POINTER(L.EmcmcUpdateDesc)).contents
        self.added.append((int(u.kernel), int(u.num_coords)))
        return L.OK

    def emcmc_last_error(self, h):
        return b""


def _host_engine(dim):
    eng = Engine.__new__(Engine)
    eng.cfg = EngineConfig(dim=dim, num_chains=4, num_mcmc_steps=10)
    eng._lib = _RecordingLib()
    eng._h = None
    eng.num_updates = 0
    eng._update_n = []
    eng._cb_error = None
    return eng


def test_add_update_desc_records_the_update_shape():
    """add_update_desc (raw descriptors, as the Julia shim passes them) keeps the
    per-update coordinate count that get_mix_state / get_adaptation_moments index by."""
    eng = _host_engine(6)
    coords = np.arange(4, dtype=np.uint32)
    u = L.EmcmcUpdateDesc()
    u.kernel = L.RW_GAUSSIAN
    u.num_coords = 4
    u.coords = L.u32ptr(coords)
    eng.add_update_desc(u)
    u2 = L.EmcmcUpdateDesc()
    u2.kernel = L.RW_UNIFORM
    u2.num_coords = 2
    eng.add_update_desc(u2)
    assert eng.num_updates == 2
    assert eng._update_n == [4, 2]
    assert eng._lib.added == [(L.RW_GAUSSIAN, 4), (L.RW_UNIFORM, 2)]
