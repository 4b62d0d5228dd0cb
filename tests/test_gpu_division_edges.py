"""The fused epilogue's division (`parameter / total_weight`, fed_avg_algorithm.py:71-74) at the
edges of its fast path (csrc/exact_div.h: one reciprocal per lane + a correction step, the IEEE
division for waves it does not cover).

Every case is compared BIT-FOR-BIT with the oracle: accumulators of ±0 (the sign of a zero
quotient), fp64 subnormals, values below 2^-900 and above 2^900, ±inf, totals below 2^-60 and
above 2^60, negative totals, and ordinary elements sharing a wave with any of them.
"""

from __future__ import annotations

import zlib

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, PersonalizedFedAVGAlgorithm
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage
from oracle.personalized_oracle import OraclePersonalizedFedAvg
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

SPECIALS = np.array([0.0, -0.0, 5e-324, -2.5e-320, 1e-300, -3e-290, 1e-271, 2e290, -7e299, np.inf, -np.inf,
                     1.0, -1.0, 2.0**-900, 2.0**900], dtype=np.float64)


def _clients(n: int, numel: int, seed: int, special_at: list[int]) -> list[np.ndarray]:
    """n clients of fp64 N(0, 1) values; at each index of `special_at` every client carries the
    same special value (so the accumulator is that value times the total, or ±0 / ±inf)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        x = rng.standard_normal(numel)
        for j, idx in enumerate(special_at):
            x[idx] = SPECIALS[j % len(SPECIALS)]
        out.append(x)
    return out


WEIGHTS = {
    "int": lambda n: [float(100 + 37 * i) for i in range(n)],
    "tiny_total": lambda n: [1e-22 * (i + 1) for i in range(n)],  # W ~ 1e-21 < 2^-60
    "huge_total": lambda n: [3e18 * (i + 1) for i in range(n)],  # W > 2^60
    "negative_total": lambda n: [-(i + 1.5) for i in range(n)],
    "mixed_sign": lambda n: [(-1) ** i * (i + 2.25) for i in range(n)],
}


@pytest.mark.parametrize("kind", list(WEIGHTS))
@pytest.mark.parametrize("special", ["none", "scattered", "one_wave"])
def test_fedavg_division_edges_bit_identical(hip_device, kind, special):
    n, numel = 5, 3 * 4096 + 77
    if special == "none":
        at = []
    elif special == "scattered":  # one special per wave-sized stretch: most waves take the fallback
        at = list(range(3, numel, 977))
    else:  # all specials inside one lane group: the other waves stay on the fast path
        at = list(range(4096 + 64, 4096 + 64 + len(SPECIALS)))
    xs = _clients(n, numel, seed=zlib.crc32(f"{kind}/{special}".encode()), special_at=at)
    weights = WEIGHTS[kind](n)
    algo = FedAVGAlgorithm(device=hip_device)
    oracle = OracleFedAvg()
    for k, (x, w) in enumerate(zip(xs, weights)):
        algo.process_worker_data(k, ParameterMessage(parameter={"t": torch.from_numpy(x).to(hip_device)},
                                                     aggregation_weight=w))
        oracle.process_worker_data(k, OracleMessage(parameter={"t": x.copy()}, aggregation_weight=w))
    try:
        want = oracle.aggregate_worker_data().parameter
    except AssertionError:  # inf - inf somewhere (mixed-sign weights on ±inf): both must raise
        with pytest.raises(AssertionError):
            algo.aggregate_worker_data()
        return
    got = algo.aggregate_worker_data().parameter
    assert bits_equal(got["t"].cpu().numpy(), want["t"])


@pytest.mark.parametrize("kind", ["int", "tiny_total", "huge_total"])
def test_personalized_division_edges_bit_identical(hip_device, kind):
    n, numel = 4, 2 * 4096 + 33
    at = list(range(5, numel, 1311))
    # no ±inf here: a receiver's fold over inf and -inf clients would be NaN in both paths anyway
    xs = [np.nan_to_num(x, posinf=1e300, neginf=-1e300) for x in _clients(n, numel, seed=7, special_at=at)]
    base = WEIGHTS[kind](n)
    ww = {j: {i: base[(i + j) % n] for i in range(n) if i != j} for j in range(n)}
    algo = PersonalizedFedAVGAlgorithm(device=hip_device)
    oracle = OraclePersonalizedFedAvg()
    algo.set_worker_weights({j: dict(v) for j, v in ww.items()})
    oracle.set_worker_weights({j: dict(v) for j, v in ww.items()})
    for k, x in enumerate(xs):
        algo.process_worker_data(k, ParameterMessage(parameter={"t": torch.from_numpy(x).to(hip_device)}))
        oracle.process_worker_data(k, OracleMessage(parameter={"t": x.copy()}))
    want = oracle.aggregate_worker_data()
    got = algo.aggregate_worker_data()
    assert list(got.worker_data) == list(want.worker_data)
    for j, r in want.worker_data.items():
        assert bits_equal(got.worker_data[j].parameter["t"].cpu().numpy(), r.parameter["t"]), j
    assert bits_equal(got.other_data["centralized_parameter"]["t"].cpu().numpy(), want.centralized_parameter["t"])
