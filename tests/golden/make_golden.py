"""Generates the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py

* philox_kat.json    — Random123 published known-answer vectors for
                       philox4x32_10 (Salmon et al., SC'11; Random123 kat_vectors).
* schedule_kat.json  — the reference's own schedule KAT, transcribed as data
                       from /root/reference/test/runtests.jl:5-32 (inputs, the
                       mid-iteration reschedule! call and the expected tuples).
* adaptation_kat.json — AdaptationUnifRW field expectations transcribed from
                       /root/reference/test/runtests.jl:34-85.
* gsn_*.npz          — oracle outputs (oracle/lib/liboracle.so) on small
                       workloads: per-step θ, θ°, ll, accept bits, final state.
                       These pin the oracle against regressions; the engine is
                       compared with the live oracle and with these files.
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "extensiblemcmc.jl_amd"))

from oracle import oracle as O  # noqa: E402
from extensible_mcmc import workloads as W  # noqa: E402

PHILOX_KAT = [
    {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
    {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
    {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
     "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
]

SCHEDULE_KAT = {
    "source": "reference test/runtests.jl:5-32",
    "num_mcmc_iter": 10,
    "num_params": 4,
    "exclude_params": [[1, [3, 8, 1]], [2, [4, 10, 2]]],
    "reschedule_at": [5, 3],
    "reschedule_args": {"num_new_updates": 2, "idxes_to_remove": [4], "idxes_to_add": [[5, [8, 9, 1]]]},
    "expected": [
        [1, 1], [1, 2], [1, 3], [1, 4],
        [2, 1], [2, 2], [2, 3], [2, 4],
        [3, 2], [3, 3], [3, 4],
        [4, 3], [4, 4],
        [5, 2], [5, 3], [5, 4], [5, 5], [5, 6],
        [6, 3], [6, 5], [6, 6],
        [7, 2], [7, 3], [7, 5], [7, 6],
        [8, 3], [8, 6],
        [9, 1], [9, 2], [9, 3], [9, 6],
        [10, 1], [10, 3], [10, 5], [10, 6],
    ],
}

ADAPTATION_KAT = {
    "source": "reference test/runtests.jl:34-85",
    "template": {"target_accpt_rate": 0.234, "adapt_every_k_steps": 100, "scale": 1.0, "min": 1e-12,
                 "max": 1e7, "offset": 1e2, "N": 1},
    "ar_vec": {"target_accpt_rate": 0.111, "min": [10.0, 10.0], "max": [1e7, 1e7], "scale": [3.0, 4.0],
               "offset": [100.0, 100.0], "N": 2, "adapt_every_k_steps": 100},
}


def gsn_fixture(w, nchains, nsteps, ll_mode, seed):
    st = O.OracleState(np.broadcast_to(w.theta_init, (nchains, w.D)).copy())
    h = O.run_gsn(st, seed=seed, rw_sigma=w.rw_sigma, t_sigma=w.t_sigma, obs=w.obs, iter0=1, nsteps=nsteps,
                  ll_mode=ll_mode, nthreads=1)
    return {
        "theta_hist": h["theta"], "prop_hist": h["prop"], "ll_hist": h["ll"], "acc_hist": h["acc"],
        "theta": st.theta, "ll": st.ll, "ra": st.ra, "nacc": st.nacc, "ring": st.ring,
        "rw_sigma": w.rw_sigma, "t_sigma": w.t_sigma, "obs": w.obs, "theta_init": np.asarray(w.theta_init),
        "seed": np.uint64(seed), "ll_mode": np.int64(ll_mode),
    }


def mwg_fixture():
    """The reference's own test workload (test/runtests.jl:87-114): two single-site
    UniformRandomWalk([1.0]) updates, 8 chains × 200 iterations, and the
    tutorial's adaptive variant (ϵ = 0.1, AdaptationUnifRW k = 50, scale = 0.1)."""
    w = W.ref_test()
    out = {"obs": np.asarray(w.obs), "t_sigma": np.asarray(w.t_sigma), "mu0": np.array([1.0, 2.0]),
           "seed": np.uint64(W.SEED)}
    steps = [(i, p) for i in range(1, 201) for p in (1, 2)]
    out["steps"] = np.asarray(steps, dtype=np.uint32)
    for tag, eps, ad in (("plain", 1.0, None),
                         ("adapt", 0.1, {"k": 50, "target": 0.234, "scale": 0.1, "min": 1e-12, "max": 1e7,
                                          "offset": 1e2})):
        ups = [O.mwg_update(1, [0], eps=[eps], adapt=ad), O.mwg_update(1, [1], eps=[eps], adapt=ad)]
        st = O.MWGState(np.zeros((8, 2)), [1.0, 2.0], ups)
        h = O.run_mwg(st, ups, seed=W.SEED, t_sigma=w.t_sigma, obs=w.obs, steps=steps)
        out[f"{tag}_acc"] = h["acc"]
        out[f"{tag}_theta"] = h["theta"]
        out[f"{tag}_ll"] = h["ll"]
        out[f"{tag}_ra"] = st.ra
        out[f"{tag}_eps"] = st.eps[:, :, 0]
    return out


def main():
    O.build()
    (HERE / "philox_kat.json").write_text(json.dumps(PHILOX_KAT, indent=1))
    (HERE / "schedule_kat.json").write_text(json.dumps(SCHEDULE_KAT, indent=1))
    (HERE / "adaptation_kat.json").write_text(json.dumps(ADAPTATION_KAT, indent=1))
    np.savez_compressed(HERE / "gsn_d2_reftest.npz", **gsn_fixture(W.ref_test(), 8, 200, 0, W.SEED))
    np.savez_compressed(HERE / "gsn_d2_iso.npz", **gsn_fixture(W.cfg1(True), 8, 200, 0, W.SEED))
    np.savez_compressed(HERE / "gsn_d32_perobs.npz", **gsn_fixture(W.cfg2(8), 8, 200, 0, W.SEED))
    np.savez_compressed(HERE / "gsn_d32_suffstat.npz", **gsn_fixture(W.cfg2(8), 8, 200, 1, W.SEED))
    np.savez_compressed(HERE / "mwg_d2_reftest.npz", **mwg_fixture())
    print("wrote", sorted(p.name for p in HERE.iterdir()))


if __name__ == "__main__":
    main()
