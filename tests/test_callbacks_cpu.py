"""SavingCallback's CSV entries as Julia writes them: `"$θₖ, "` interpolates
string(::Float64) (callbacks.jl:249-253), Julia's shortest round-trip form
(Base.Ryu.writeshortest).  Expected strings are Julia's documented printing of
these values (no Julia in the image to regenerate them: parity unpinned beyond
the rules restated in callbacks.julia_float_string)."""
import numpy as np
import pytest

from extensible_mcmc.callbacks import _fmt, julia_float_string

CASES = [
    (1e-5, "1.0e-5"), (1.5e-7, "1.5e-7"), (1e-4, "0.0001"), (0.000123, "0.000123"), (1e6, "1.0e6"),
    (1e5, "100000.0"), (123456.7, "123456.7"), (1234567.8, "1.2345678e6"), (-2.5, "-2.5"), (1.0, "1.0"),
    (0.1, "0.1"), (0.1 + 0.2, "0.30000000000000004"), (1e300, "1.0e300"), (5e-324, "5.0e-324"),
    (-0.0, "-0.0"), (0.0, "0.0"), (float("nan"), "NaN"), (float("inf"), "Inf"), (-float("inf"), "-Inf"),
    (-1.3241e-10, "-1.3241e-10"), (2.0, "2.0"), (1e15, "1.0e15"),
]


@pytest.mark.parametrize("x,s", CASES)
def test_julia_float_string(x, s):
    assert julia_float_string(x) == s


def test_round_trip_and_bools():
    rng = np.random.default_rng(3)
    for x in np.concatenate([rng.standard_normal(2000) * 10.0 ** rng.integers(-12, 12, 2000), [np.pi, -np.e]]):
        assert float(julia_float_string(x)) == x
    assert _fmt(True) == "true" and _fmt(np.bool_(False)) == "false"
