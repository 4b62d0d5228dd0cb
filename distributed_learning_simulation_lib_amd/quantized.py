"""Quantised client updates, dequantised inside the FedAvg fold on the GPU.

The reference can run its workers behind ``StochasticQuantClientEndpoint`` and the server behind
``StochasticQuantServerEndpoint`` (simulation_lib/topology/quantized_endpoint.py:96-111): every
parameter tensor travels QSGD-quantised at ``quantization_level=255`` (one norm per tensor, a
uint8 slot and a sign bit per element) and ``QuantServerEndpoint.get`` (:69-77) dequantises it
on the host before the FedAvg algorithm folds the dense copy (fed_avg_algorithm.py:43-64).

Here the quantised tensor itself is the client operand. A ``QuantizedTensor`` is one record in
the layout of ``include/fedavg_hip.h`` (FEDAVG_QSGD_F32): a 16-byte header (norm, level), the
slots, the packed sign bits. ``FedAVGAlgorithm`` passes record pointers to the kernels with the
``QSGD_F32`` / ``QSGD_F64`` input format and the kernel folds ``round(f64(x_hat) * w)`` per
element with x_hat = ((norm * sign) * slot) / level computed in the codec's dtype — the same
value the host dequantisation would have produced — while reading 1.125 bytes per element
instead of 4 or 8.

The codec is the unvendored ``cyy_torch_algorithm.quantization.stochastic`` (git ``@main``);
it is restated from the published QSGD scheme, so parity with it is unpinned
(``oracle/qsgd_oracle.py`` says what exactly is claimed). ``stochastic_quantization`` below is
this framework's client-side quantiser (and a host dequantiser for consumers that need dense
tensors, e.g. workers receiving a quantised broadcast); the server-side hot path never calls
``dequantize_tensor``.
"""

from __future__ import annotations

from collections.abc import Callable, Mapping
from dataclasses import dataclass

import torch

from . import _native
from .fedavg import ModelLayout

HEADER_BYTES = 16
DEFAULT_LEVEL = 255  # quantized_endpoint.py:104,110


@dataclass(frozen=True)
class QuantizedDtype:
    """Input format code of quantised records for the C ABI (``fedavg_dtype``)."""

    name: str
    value_dtype: torch.dtype  # the codec's arithmetic dtype (what dequant returns)
    code: int


QSGD_F32 = QuantizedDtype("qsgd_f32", torch.float32, _native.QSGD_F32)
QSGD_F64 = QuantizedDtype("qsgd_f64", torch.float64, _native.QSGD_F64)


def codec_for(dtype: torch.dtype) -> QuantizedDtype:
    return QSGD_F64 if dtype == torch.float64 else QSGD_F32


def _align16(n: int) -> int:
    return (n + 15) // 16 * 16


def sign_offset(numel: int) -> int:
    """Byte offset of the sign bits in a record (== fedavg_qsgd_sign_offset)."""
    return HEADER_BYTES + _align16(numel)


def record_bytes(numel: int) -> int:
    """Byte size of one record (== fedavg_qsgd_record_bytes)."""
    return sign_offset(numel) + _align16((numel + 7) // 8)


@dataclass
class QuantizedTensor:
    """One QSGD-quantised parameter tensor: a record (uint8, 1-D) + its shape and codec."""

    record: torch.Tensor
    shape: tuple[int, ...]
    codec: QuantizedDtype

    def __post_init__(self) -> None:
        self.shape = tuple(int(s) for s in self.shape)
        if self.record.dtype != torch.uint8 or self.record.dim() != 1:
            raise ValueError("a QSGD record is a 1-D uint8 tensor")
        if self.record.numel() != record_bytes(self.numel):
            raise ValueError(f"record holds {self.record.numel()} bytes, the layout needs {record_bytes(self.numel)}")

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n

    @property
    def device(self) -> torch.device:
        return self.record.device

    @property
    def dtype(self) -> torch.dtype:
        return self.codec.value_dtype

    @property
    def norm(self) -> float:
        return float(self.record[0:8].cpu().view(torch.float64)[0])

    @property
    def level(self) -> int:
        return int(self.record[8:12].cpu().view(torch.int32)[0])

    @property
    def slots(self) -> torch.Tensor:
        return self.record[HEADER_BYTES : HEADER_BYTES + self.numel]

    @property
    def sign_bits(self) -> torch.Tensor:
        """One 0/1 (uint8) per element, 1 = non-negative."""
        so = sign_offset(self.numel)
        packed = self.record[so : so + (self.numel + 7) // 8]
        shifts = torch.arange(7, -1, -1, device=packed.device, dtype=torch.uint8)
        return ((packed.unsqueeze(1) >> shifts) & 1).reshape(-1)[: self.numel]

    def to(self, device: torch.device | str, non_blocking: bool = False) -> QuantizedTensor:
        return QuantizedTensor(self.record.to(device, non_blocking=non_blocking), self.shape, self.codec)


_BIT_WEIGHTS: dict[torch.device, torch.Tensor] = {}


def _pack_bits(bits: torch.Tensor) -> torch.Tensor:
    """numpy.packbits order: element i -> byte i // 8, bit 7 - i % 8 (zero padded)."""
    n = bits.numel()
    pad = (-n) % 8
    b = bits.to(torch.uint8)
    if pad:
        b = torch.cat([b, torch.zeros(pad, dtype=torch.uint8, device=b.device)])
    w = _BIT_WEIGHTS.get(b.device)
    if w is None:
        w = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.int32, device=b.device)
        _BIT_WEIGHTS[b.device] = w
    return (b.view(-1, 8).to(torch.int32) * w).sum(dim=1).to(torch.uint8)


def quantize_tensor(
    tensor: torch.Tensor,
    quantization_level: int = DEFAULT_LEVEL,
    use_l2_norm: bool = False,
    generator: torch.Generator | None = None,
) -> QuantizedTensor:
    """QSGD quantisation of one tensor (on its own device): norm n = max|x| (l2 if asked),
    r = |x| / n * level, slot = floor(r) + Bernoulli(r - floor(r)), sign bit = not (x < 0)."""
    if not 1 <= quantization_level <= 255:
        raise ValueError("quantization_level must be in [1, 255] (one byte per slot)")
    codec = codec_for(tensor.dtype)
    v = tensor.detach().reshape(-1).to(codec.value_dtype)
    n = v.numel()
    dev = v.device
    rec = torch.zeros(record_bytes(n), dtype=torch.uint8, device=dev)
    if n:
        absv = v.abs()
        norm = torch.linalg.vector_norm(v) if use_l2_norm else absv.max()
        r = (absv / norm) * quantization_level
        fl = torch.floor(r)
        u = torch.rand(n, generator=generator, device=dev, dtype=codec.value_dtype)
        slots = fl + (u < (r - fl)).to(fl.dtype)
        slots = torch.where(norm > 0, slots, torch.zeros_like(slots))
        slots = slots.clamp_(0, quantization_level).to(torch.uint8)
        rec[HEADER_BYTES : HEADER_BYTES + n] = slots
        packed = _pack_bits(~(v < 0))
        so = sign_offset(n)
        rec[so : so + packed.numel()] = packed
        rec[0:8] = norm.to(torch.float64).reshape(1).view(torch.uint8)
    rec[8:12] = torch.tensor([quantization_level], dtype=torch.int32).view(torch.uint8).to(dev)
    return QuantizedTensor(rec, tuple(tensor.shape), codec)


def dequantize_tensor(q: QuantizedTensor) -> torch.Tensor:
    """Dense x_hat = ((norm * sign) * slot) / level in the codec's dtype (host-side consumers;
    the server's FedAvg fold dequantises inside the kernel instead)."""
    dt = q.codec.value_dtype
    rec = q.record
    norm = rec[0:8].view(torch.float64).to(dt)
    level = rec[8:12].view(torch.int32).to(dt)
    sign = q.sign_bits.to(dt) * 2 - 1
    x = (norm * sign) * q.slots.to(dt)
    return (x / level).reshape(q.shape)  # tensor / tensor: a true division, never a reciprocal


def stochastic_quantization(
    quantization_level: int = DEFAULT_LEVEL,
    use_l2_norm: bool = False,
    generator: torch.Generator | None = None,
) -> tuple[Callable[[Mapping[str, torch.Tensor]], dict[str, QuantizedTensor]],
           Callable[[Mapping[str, QuantizedTensor]], dict[str, torch.Tensor]]]:
    """The (quant, dequant) pair the reference's endpoints take (quantized_endpoint.py:96-111)."""

    def quant(parameter: Mapping[str, torch.Tensor]) -> dict[str, QuantizedTensor]:
        return {k: quantize_tensor(v, quantization_level, use_l2_norm, generator) for k, v in parameter.items()}

    def dequant(parameter: Mapping[str, QuantizedTensor]) -> dict[str, torch.Tensor]:
        return {k: dequantize_tensor(v) if isinstance(v, QuantizedTensor) else v for k, v in parameter.items()}

    return quant, dequant


def is_quantized(parameter: Mapping[str, object]) -> bool:
    return any(isinstance(v, QuantizedTensor) for v in parameter.values())


def dequantize_parameter(parameter: Mapping[str, object]) -> dict[str, object]:
    """QuantServerEndpoint.get's dequantisation (quantized_endpoint.py:69-77) for consumers
    that cannot take records (the fused FedAvg path never calls this)."""
    return {k: dequantize_tensor(v) if isinstance(v, QuantizedTensor) else v for k, v in parameter.items()}


def record_layout(numels: list[int]) -> ModelLayout:
    """Byte layout of one client's records in one bucket (every record 16-B aligned)."""
    return ModelLayout(names=tuple(f"r{i}" for i in range(len(numels))),
                       shapes=tuple((record_bytes(n),) for n in numels))
