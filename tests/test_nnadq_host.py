"""Host logic of the NNADQ path (no GPU): the record format, the client-side quantiser and the
host dequantiser against the oracle restatement, the C library's record geometry, the level
choice's edges, and the endpoint pair (quantized_endpoint.py:114-142).

Parity note: the codec is the unvendored cyy_torch_algorithm (git @main,
quantization.deterministic); oracle/nnadq_oracle.py restates a deterministic adaptive-level
affine code, so these checks pin this framework's codec to that restatement, not to
cyy_torch_algorithm ("parity unpinned").
"""

from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import _native
from distributed_learning_simulation_lib_amd.message import ParameterMessage
from distributed_learning_simulation_lib_amd.quantized import (
    NNADQ,
    NNADQ_F32,
    NNADQ_F64,
    NeuralNetworkAdaptiveDeterministicQuant,
    QuantizedTensor,
    codec_for,
    dequantize_tensor,
    nnadq_levels,
    nnadq_quantize_tensor,
)
from distributed_learning_simulation_lib_amd.server import AggregationServer
from oracle import nnadq_oracle as no

SIZES = [0, 1, 7, 15, 16, 17, 255, 4095, 4096, 4097, 10_000]


@pytest.mark.parametrize("n", SIZES)
def test_record_geometry_matches_oracle_and_library(n):
    lib = _native.load()
    assert NNADQ_F32.record_bytes(n) == no.record_bytes(n) == lib.fedavg_nnadq_record_bytes(n)
    assert no.record_bytes(n) % 16 == 0
    assert lib.fedavg_nnadq_record_bytes(-1) == -1


def test_codec_selection():
    assert codec_for(torch.float64, "nnadq") is NNADQ_F64
    for dt in (torch.float32, torch.float16, torch.bfloat16):
        assert codec_for(dt, "nnadq") is NNADQ_F32
    assert NNADQ_F32.code == _native.NNADQ_F32 and NNADQ_F64.code == _native.NNADQ_F64


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.float16])
@pytest.mark.parametrize("n", [1, 9, 4097])
@pytest.mark.parametrize("weight", [0.001, 0.01, 0.5])
def test_torch_quantiser_equals_oracle_record(dtype, n, weight):
    """The framework's quantiser and the oracle's produce the same record, byte for byte."""
    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, generator=g, dtype=torch.float64) * 3.0).to(dtype)
    q = nnadq_quantize_tensor(x, weight)
    codec_np = np.float64 if dtype == torch.float64 else np.float32
    want = no.quantize(x.to(torch.float64 if dtype == torch.float64 else torch.float32).numpy().astype(codec_np),
                       weight)
    assert q.codec is codec_for(dtype, "nnadq") and q.shape == (n,)
    assert np.array_equal(q.record.numpy(), want)
    lo, step, levels, codes = no.parse(want, n)
    assert (q.lo, q.step, q.levels) == (lo, step, levels)
    assert np.array_equal(q.codes.numpy(), codes)
    assert 1 <= levels <= 255 and int(codes.max()) <= levels


@pytest.mark.parametrize("codec", ["float32", "float64"])
def test_host_dequantiser_bit_identical_to_oracle(codec):
    rng = np.random.default_rng(5)
    for n in [1, 13, 4096, 5000]:
        x = (rng.standard_normal(n) * rng.choice([1e-3, 1.0, 7e3])).astype(codec)
        rec = no.quantize(x, float(rng.choice([0.002, 0.05])))
        q = QuantizedTensor(torch.from_numpy(rec), (n,), NNADQ_F64 if codec == "float64" else NNADQ_F32)
        got = dequantize_tensor(q).numpy()
        want = no.dequantize(rec, n, codec)
        assert got.dtype == want.dtype
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_error_bound():
    """|x - x_hat| <= step / 2 (+ the two roundings of the dequantisation)."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(5000, generator=g, dtype=torch.float64)
    for weight in (0.001, 0.01, 0.1):
        q = nnadq_quantize_tensor(x, weight)
        xh = dequantize_tensor(q)
        assert float((x - xh).abs().max()) <= q.step / 2 * (1 + 1e-9) + 4 * np.finfo(np.float64).eps * float(x.abs().max())
        # the step never exceeds weight x the largest magnitude unless the 255-level cap binds
        amax = float(x.abs().max())
        assert q.levels == 255 or q.step <= weight * amax * (1 + 1e-12)


@pytest.mark.parametrize(
    "lo,hi,weight,want",
    [
        (0.0, 0.0, 0.01, 1),  # constant zero tensor
        (2.0, 2.0, 0.01, 1),  # constant tensor: range 0
        (-1.0, 1.0, 0.01, 200),  # (hi - lo) / (w * amax) = 200
        (-1.0, 1.0, 0.001, 255),  # 2000 levels asked: capped
        (-1.0, 1.0, 1.0, 2),
        (-1.0, 1.0, 5.0, 1),  # coarser than the range: one level
        (-1.0, 1.0, 0.0, 1),  # no weight
        (float("nan"), 1.0, 0.01, 1),  # NaN tensor: codes 0, dequantised NaN (lo NaN)
        (-float("inf"), 1.0, 0.01, 1),
    ],
)
def test_level_choice_edges(lo, hi, weight, want):
    assert nnadq_levels(lo, hi, weight) == no.choose_levels(lo, hi, weight) == want


def test_constant_and_empty_tensors():
    for v in (0.0, -3.5):
        q = nnadq_quantize_tensor(torch.full((33,), v), 0.01)
        assert q.step == 0.0 and q.levels == 1 and int(q.codes.sum()) == 0
        assert torch.equal(dequantize_tensor(q), torch.full((33,), v))
    q = nnadq_quantize_tensor(torch.zeros(0), 0.01)
    assert q.numel == 0 and q.record.numel() == no.record_bytes(0)


def test_nan_tensor_dequantises_to_nan():
    x = torch.randn(40)
    x[7] = float("nan")
    q = nnadq_quantize_tensor(x, 0.01)
    assert math.isnan(q.lo)
    assert torch.isnan(dequantize_tensor(q)).all()
    assert np.isnan(no.dequantize(q.record.numpy(), 40, "float32")).all()


def test_endpoint_pair_and_compression_ratio():
    quant, dequant = NNADQ(weight=0.01)
    g = torch.Generator().manual_seed(1)
    p = {"w": torch.randn(64, 9, generator=g), "b": torch.randn(64, generator=g)}
    q = quant(p)
    assert all(isinstance(v, QuantizedTensor) and v.codec is NNADQ_F32 for v in q.values())
    back = dequant(q)
    for k, v in p.items():
        assert back[k].shape == v.shape and back[k].dtype == torch.float32
        assert float((back[k] - v).abs().max()) <= q[k].step / 2 * (1 + 1e-6) + 1e-6
    ratio = NeuralNetworkAdaptiveDeterministicQuant.check_compression_ratio(ParameterMessage(parameter=q))
    dense = sum(v.numel() * 4 for v in p.values())
    assert ratio == pytest.approx(sum(v.record.numel() for v in q.values()) / dense)
    assert ratio < 0.4


class _Recorder:
    def __init__(self) -> None:
        self.seen = []

    def set_config(self, config) -> None:
        pass

    def process_worker_data(self, worker_id, worker_data) -> bool:
        self.seen.append(worker_data)
        return True


class _FusedRecorder(_Recorder):
    accepts_quantized_messages = True


def test_server_dequantises_nnadq_unless_the_algorithm_fuses():
    quant, _ = NNADQ(weight=0.01)
    x = {"w": torch.randn(33), "b": torch.randn(4)}
    for algo_cls, expect_records in [(_Recorder, False), (_FusedRecorder, True)]:
        algo = algo_cls()
        srv = AggregationServer(algorithm=algo, worker_number=2, endpoint=None)
        srv._process_worker_data(0, ParameterMessage(parameter=quant(x), aggregation_weight=1.0))
        got = algo.seen[0].parameter
        assert all(isinstance(v, QuantizedTensor) == expect_records for v in got.values())
        if not expect_records:
            want = no.dequantize(quant(x)["w"].record.numpy(), 33, "float32")
            assert np.array_equal(got["w"].numpy().view(np.uint32), want.view(np.uint32))
