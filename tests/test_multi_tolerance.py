"""CPU: the multi-device composition (entry-ordered sum of per-entry chains, what the peer exchange
computes bit for bit) stays within the stated tolerance of the reference's single chain on every
golden case — the bound the GPU tests assert on the device results (tests/test_gpu_multi_device.py)."""

from __future__ import annotations

import numpy as np
import pytest

from tests.golden_io import load_golden
from tests.multi_tolerance import reference_magnitude, sharded_expectation, within_reference_tolerance

CASES = load_golden()
ACCUMULATING = sorted(n for n, c in CASES.items() if c.error is None and c.accumulate)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("name", ACCUMULATING)
def test_sharded_composition_within_tolerance_of_the_reference(name, world):
    case = CASES[name]
    got = sharded_expectation(case, world)
    mag = reference_magnitude(case)
    assert list(got) == list(case.expected)
    for k, want in case.expected.items():
        ok, why = within_reference_tolerance(got[k], want, mag[k])
        assert ok, f"{name}/{k}: {why}"


def test_the_tolerance_rejects_a_two_ulp_error():
    case = CASES["n64_f32"] if "n64_f32" in CASES else CASES[ACCUMULATING[0]]
    mag = reference_magnitude(case)
    k = next(iter(case.expected))
    want = case.expected[k]
    bad = want.astype(np.float32)
    flat = bad.reshape(-1)
    flat[0] = np.nextafter(np.nextafter(flat[0], np.float32(np.inf)), np.float32(np.inf))
    ok, why = within_reference_tolerance(bad.astype(np.float64), want, mag[k])
    assert not ok
