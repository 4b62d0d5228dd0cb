"""Property tests (hypothesis) of the HIP paths against the oracle, on the MI355X.

Random client counts, layouts (segment sizes that are not multiples of any vector width, tiny
and multi-tile segments), input dtypes, weight kinds (integer: fused fold; fractional: rounded
mul + add; zeros), skipped clients, missing tensors and wave sizes. Tolerance: none — every
result is compared BIT-FOR-BIT with the oracle (itself pinned to the reference's own outputs,
tests/test_oracle_golden.py, tests/test_oracle_personalized.py).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, PersonalizedFedAVGAlgorithm
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage
from oracle.personalized_oracle import OraclePersonalizedFedAvg
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu
SETTINGS = settings(max_examples=60, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
TORCH_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64}


def _np(t: torch.Tensor) -> np.ndarray:
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def _weights(rng, kind, n):
    if kind == "int":
        return [int(x) for x in rng.integers(1, 5000, size=n)]
    if kind == "zeros_some":
        return [0 if i % 3 == 1 else float(rng.uniform(0.1, 3.0)) for i in range(n)]
    return [float(x) for x in rng.uniform(1e-3, 10.0, size=n)]


@SETTINGS
@given(n=st.integers(1, 24), sizes=st.lists(st.integers(1, 9000), min_size=1, max_size=5),
       dtype=st.sampled_from(list(TORCH_DT)), kind=st.sampled_from(["int", "float", "zeros_some"]),
       wave=st.integers(1, 30), seed=st.integers(0, 2**31 - 1), skip_every=st.integers(0, 5),
       drop_key=st.booleans())
def test_fedavg_random_rounds_are_bit_identical(hip_device, n, sizes, dtype, kind, wave, seed, skip_every, drop_key):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    shapes = {f"t{i}": (s,) for i, s in enumerate(sizes)}
    weights = _weights(rng, kind, n)
    if sum(weights) == 0:
        weights[0] = 1
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave)
    oracle = OracleFedAvg()
    first = True
    for k in range(n):
        if skip_every and k % skip_every == skip_every - 1 and k != 0:
            algo.process_worker_data(k, None)
            oracle.process_worker_data(k, None)
            continue
        p = {name: torch.randn(s, generator=g).to(TORCH_DT[dtype]) for name, s in shapes.items()}
        if drop_key and not first and len(shapes) > 1 and k % 2 == 1:
            del p[f"t{len(sizes) - 1}"]  # a later client without the last tensor
        first = False
        algo.process_worker_data(k, ParameterMessage(parameter={a: b.to(hip_device) for a, b in p.items()},
                                                     aggregation_weight=weights[k]))
        oracle.process_worker_data(k, OracleMessage(parameter={a: _np(b) for a, b in p.items()},
                                                    aggregation_weight=weights[k],
                                                    dtype="bfloat16" if dtype == "bfloat16" else None))
    try:
        want = oracle.aggregate_worker_data().parameter
    except AssertionError:  # e.g. the only client carrying a tensor had weight 0: 0/0
        with pytest.raises(AssertionError):
            algo.aggregate_worker_data()
        return
    got = algo.aggregate_worker_data().parameter
    assert list(got) == list(want)
    for name, w in want.items():
        assert bits_equal(got[name].cpu().numpy(), w), name


@SETTINGS
@given(workers=st.integers(2, 60), n_recv=st.integers(1, 60), sizes=st.lists(st.integers(1, 3000), min_size=1, max_size=3),
       dtype=st.sampled_from(list(TORCH_DT)), kind=st.sampled_from(["int", "float", "sparse"]),
       seed=st.integers(0, 2**31 - 1), skip=st.integers(-1, 19))
def test_personalized_random_rounds_are_bit_identical(hip_device, workers, n_recv, sizes, dtype, kind, seed, skip):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    receivers = [int(j) for j in rng.permutation(workers)[: min(n_recv, workers)]]
    ww = {}
    for j in receivers:
        row = {}
        for i in range(workers):
            if i == j or (kind == "sparse" and rng.random() < 0.3):
                continue
            row[i] = int(rng.integers(1, 500)) if kind == "int" else float(rng.uniform(0.01, 3.0))
        ww[j] = row
    shapes = {f"t{i}": (s,) for i, s in enumerate(sizes)}
    algo = PersonalizedFedAVGAlgorithm(device=hip_device)
    oracle = OraclePersonalizedFedAvg()
    algo.set_worker_weights({j: dict(v) for j, v in ww.items()})
    oracle.set_worker_weights({j: dict(v) for j, v in ww.items()})
    for i in rng.permutation(workers):
        i = int(i)
        if i == skip:
            algo.process_worker_data(i, None)
            oracle.process_worker_data(i, None)
            continue
        p = {name: torch.randn(s, generator=g).to(TORCH_DT[dtype]) for name, s in shapes.items()}
        algo.process_worker_data(i, ParameterMessage(parameter={a: b.to(hip_device) for a, b in p.items()}))
        oracle.process_worker_data(i, OracleMessage(parameter={a: _np(b) for a, b in p.items()},
                                                    dtype="bfloat16" if dtype == "bfloat16" else None))
    try:
        want = oracle.aggregate_worker_data()
    except AssertionError:  # a receiver with zero total weight or without any update
        with pytest.raises(AssertionError):
            algo.aggregate_worker_data()
        return
    got = algo.aggregate_worker_data()
    assert list(got.worker_data) == list(want.worker_data)
    for j, r in want.worker_data.items():
        for name, w in r.parameter.items():
            assert bits_equal(got.worker_data[j].parameter[name].cpu().numpy(), w), (j, name)
    for name, w in want.centralized_parameter.items():
        assert bits_equal(got.other_data["centralized_parameter"][name].cpu().numpy(), w), name
