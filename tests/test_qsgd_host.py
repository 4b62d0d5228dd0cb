"""Host logic of the quantised-update path (no GPU): the QSGD record format, the client-side
quantiser and the host dequantiser against the oracle restatement, the C library's record
geometry, and the server's dequantise-unless-fused rule.

Parity note: the codec is the unvendored cyy_torch_algorithm (git @main); oracle/qsgd_oracle.py
restates the published QSGD scheme, so these checks pin this framework's codec to that
restatement, not to cyy_torch_algorithm ("parity unpinned").
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import _native
from distributed_learning_simulation_lib_amd.message import DeltaParameterMessage, ParameterMessage
from distributed_learning_simulation_lib_amd.quantized import (
    QSGD_F32,
    QSGD_F64,
    QuantizedTensor,
    dequantize_tensor,
    quantize_tensor,
    record_bytes,
    sign_offset,
    stochastic_quantization,
)
from distributed_learning_simulation_lib_amd.server import AggregationServer
from oracle import qsgd_oracle as qo

SIZES = [0, 1, 7, 8, 9, 15, 16, 17, 255, 4095, 4096, 4097, 10_000]


@pytest.mark.parametrize("n", SIZES)
def test_record_geometry_matches_oracle_and_library(n):
    lib = _native.load()
    assert record_bytes(n) == qo.record_bytes(n) == lib.fedavg_qsgd_record_bytes(n)
    assert sign_offset(n) == qo.sign_offset(n) == lib.fedavg_qsgd_sign_offset(n)
    assert record_bytes(n) % 16 == 0 and sign_offset(n) % 16 == 0
    assert lib.fedavg_qsgd_record_bytes(-1) == -1


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.float16])
@pytest.mark.parametrize("n", [1, 9, 4097])
def test_torch_quantiser_fields(dtype, n):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g, dtype=torch.float64).to(dtype)
    if n > 1:
        x[0] = -0.0
    q = quantize_tensor(x, generator=g)
    codec = QSGD_F64 if dtype == torch.float64 else QSGD_F32
    assert q.codec == codec and q.shape == (n,) and q.level == 255
    norm, level, slots, bits = qo.parse(q.record.numpy(), n)
    v = x.to(codec.value_dtype).numpy()
    assert norm == float(np.max(np.abs(v)))
    assert level == 255
    r = (np.abs(v) / np.asarray(norm, dtype=v.dtype)) * v.dtype.type(255)
    assert np.all((slots == np.floor(r)) | (slots == np.ceil(r)))
    assert np.array_equal(bits, (~(v < 0)).astype(np.uint8))  # -0.0 counts as non-negative
    assert np.array_equal(q.slots.numpy(), slots) and np.array_equal(q.sign_bits.numpy(), bits)


def test_sign_bits_are_numpy_packbits_order():
    bits = np.random.default_rng(3).integers(0, 2, size=37).astype(np.uint8)
    rec = qo.make_record(1.0, 255, np.zeros(37, np.uint8), bits)
    so = qo.sign_offset(37)
    assert np.array_equal(rec[so : so + 5], np.packbits(bits))
    q = QuantizedTensor(torch.from_numpy(rec), (37,), QSGD_F32)
    assert np.array_equal(q.sign_bits.numpy(), bits)


@pytest.mark.parametrize("codec", ["float32", "float64"])
def test_host_dequantiser_bit_identical_to_oracle(codec):
    rng = np.random.default_rng(11)
    for n in [1, 13, 4096, 5000]:
        x = rng.standard_normal(n).astype(codec) * rng.choice([1e-3, 1.0, 7e3])
        rec = qo.quantize(x, rng)
        q = QuantizedTensor(torch.from_numpy(rec), (n,), QSGD_F64 if codec == "float64" else QSGD_F32)
        got = dequantize_tensor(q).numpy()
        want = qo.dequantize(rec, n, codec)
        assert got.dtype == want.dtype
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_quantiser_error_bound_and_unbiased():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2000, generator=g)
    quant, dequant = stochastic_quantization(generator=g)
    draws = torch.stack([dequant(quant({"x": x}))["x"] for _ in range(200)])
    norm = x.abs().max()
    assert torch.all((draws - x).abs() <= norm / 255 * (1 + 1e-6))
    # E[x_hat] = x: the mean over 200 draws is within a few standard errors
    se = norm / 255 / 2 / np.sqrt(200)
    assert (draws.mean(0) - x).abs().max() < 6 * se


def test_all_zero_tensor_quantises_to_zero_slots():
    q = quantize_tensor(torch.zeros(10))
    assert q.norm == 0.0 and int(q.slots.sum()) == 0
    assert torch.equal(dequantize_tensor(q), torch.zeros(10))


def test_bad_record_rejected():
    with pytest.raises(ValueError):
        QuantizedTensor(torch.zeros(10, dtype=torch.uint8), (4,), QSGD_F32)
    with pytest.raises(ValueError):
        quantize_tensor(torch.ones(3), quantization_level=256)


class _Recorder:
    """An algorithm that takes dense tensors only (no accepts_quantized_messages)."""

    def __init__(self) -> None:
        self.seen = []

    def set_config(self, config) -> None:
        pass

    def process_worker_data(self, worker_id, worker_data) -> bool:
        self.seen.append(worker_data)
        return True


class _FusedRecorder(_Recorder):
    accepts_quantized_messages = True


def test_server_dequantises_unless_the_algorithm_fuses():
    quant, _ = stochastic_quantization(generator=torch.Generator().manual_seed(1))
    x = {"w": torch.randn(33), "b": torch.randn(4)}
    for algo_cls, expect_records in [(_Recorder, False), (_FusedRecorder, True)]:
        algo = algo_cls()
        srv = AggregationServer(algorithm=algo, worker_number=2, endpoint=None)
        srv._process_worker_data(0, ParameterMessage(parameter=quant(x), aggregation_weight=1.0))
        got = algo.seen[0].parameter
        assert all(isinstance(v, QuantizedTensor) == expect_records for v in got.values())
        if not expect_records:
            assert got["w"].dtype == torch.float32 and got["w"].shape == (33,)
    # quantised deltas are always dequantised (the delta fold takes dense tensors)
    algo = _FusedRecorder()
    srv = AggregationServer(algorithm=algo, worker_number=2, endpoint=None)
    srv._model_cache.cache_parameter({k: v.double() for k, v in x.items()})
    srv._algorithm.accepts_delta_messages = True
    srv._algorithm.set_old_parameter = lambda p: None
    srv._process_worker_data(1, DeltaParameterMessage(delta_parameter=quant(x), aggregation_weight=1.0))
    assert all(isinstance(v, torch.Tensor) for v in algo.seen[0].delta_parameter.values())
