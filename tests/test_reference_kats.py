"""The reference's own known-answer tests, restated against the host mirror
(test/runtests.jl:5-85, transcribed as data in tests/golden/*.json)."""
import json

import numpy as np

from extensible_mcmc import AdaptationUnifRW, JRange, MCMCSchedule, isequal_except, reschedule


def _jr(t):
    return JRange(t[0], t[1], t[2])


def test_schedule_kat(golden_dir):
    k = json.loads((golden_dir / "schedule_kat.json").read_text())
    sched = MCMCSchedule(k["num_mcmc_iter"], k["num_params"], [(i, _jr(r)) for i, r in k["exclude_params"]])
    got = []
    ra = k["reschedule_args"]
    for s in sched:
        got.append([s.mcmciter, s.pidx])
        if [s.mcmciter, s.pidx] == k["reschedule_at"]:
            reschedule(sched, ra["num_new_updates"], ra["idxes_to_remove"],
                       [(i, _jr(r)) for i, r in ra["idxes_to_add"]])
    assert got == k["expected"]


def test_schedule_first_state_unchecked_and_plain():
    # start state is yielded without an exclusion check (schedule.jl:57,65)
    s = MCMCSchedule(3, 1, [(1, JRange(1, 1))])
    assert [(x.mcmciter, x.pidx) for x in s] == [(1, 1), (2, 1), (3, 1)]
    s = MCMCSchedule(3, 2)
    assert s.steps() == [(1, 1), (1, 2), (2, 1), (2, 2), (3, 1), (3, 2)]
    # prev_* fields carry the previous state (schedule.jl:58-63)
    steps = list(MCMCSchedule(2, 2))
    assert steps[0].prev_mcmciter is None
    assert (steps[1].prev_mcmciter, steps[1].prev_pidx) == (1, 1)


def test_adaptation_unif_rw_kat(golden_dir):
    k = json.loads((golden_dir / "adaptation_kat.json").read_text())
    t = k["template"]
    template = AdaptationUnifRW.raw(t["target_accpt_rate"], t["adapt_every_k_steps"], t["scale"], t["min"],
                                    t["max"], t["offset"], t["N"])
    assert template == AdaptationUnifRW(1.0)
    assert template == AdaptationUnifRW([2.0])
    assert template == AdaptationUnifRW(np.array([3.0]), static=True)  # SVector{1}(3.0): scalar category

    longer = AdaptationUnifRW([1.0, 2.0])
    assert template != longer
    assert isequal_except(template, longer, "N")

    longer_static = AdaptationUnifRW([1.0, 2.0, 3.0], static=True)
    assert template != longer_static
    assert isequal_except(template, longer_static, "N")

    new_scale = AdaptationUnifRW(1.0, scale=3.0)
    assert template != new_scale
    assert isequal_except(template, new_scale, "scale")

    new_params = AdaptationUnifRW(1.0, scale=3.0, target_accpt_rate=0.111, min=10.0)
    assert isequal_except(template, new_params, "scale", "target_accpt_rate", "min")
    assert new_params.scale == 3.0 and new_params.target_accpt_rate == 0.111 and new_params.min == 10.0

    e = k["ar_vec"]
    ar_vec = AdaptationUnifRW([1.0, 2.0], scale=[3.0, 4.0], target_accpt_rate=0.111, min=10.0)
    assert ar_vec.target_accpt_rate == e["target_accpt_rate"]
    assert list(ar_vec.min) == e["min"] and list(ar_vec.max) == e["max"]
    assert list(ar_vec.scale) == e["scale"] and list(ar_vec.offset) == e["offset"]
    assert ar_vec.N == e["N"] and ar_vec.adapt_every_k_steps == e["adapt_every_k_steps"]
    assert ar_vec == AdaptationUnifRW([1.0, 2.0], scale=[3.0, 4.0], target_accpt_rate=0.111, min=[10.0, 10.0])

    ar_svec = AdaptationUnifRW([1.0, 2.0], static=True, scale=[3.0, 4.0], target_accpt_rate=0.111, min=10.0)
    assert list(ar_svec.min) == e["min"] and list(ar_svec.max) == e["max"] and ar_svec.N == 2
    ar_svec2 = AdaptationUnifRW([1.0, 2.0], static=True, scale=[3.0, 4.0], target_accpt_rate=0.111,
                                min=[10.0, 10.0])
    assert ar_svec == ar_svec2
    assert ar_svec != ar_vec  # SVector{2} vs Vector element types differ (adaptation.jl:207)
