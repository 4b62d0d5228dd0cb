"""Quantised client updates, dequantised inside the FedAvg fold on the GPU.

The reference can run its workers behind ``StochasticQuantClientEndpoint`` and the server behind
``StochasticQuantServerEndpoint`` (simulation_lib/topology/quantized_endpoint.py:96-111): every
parameter tensor travels QSGD-quantised at ``quantization_level=255`` (one norm per tensor, a
uint8 slot and a sign bit per element) and ``QuantServerEndpoint.get`` (:69-77) dequantises it
on the host before the FedAvg algorithm folds the dense copy (fed_avg_algorithm.py:43-64). The
same file's ``NNADQClientEndpoint`` / ``NNADQServerEndpoint`` (:114-142) do the same with the
deterministic NNADQ codec (one lo / step per tensor, a uint8 code per element).

Here the quantised tensor itself is the client operand. A ``QuantizedTensor`` is one record in
the layout of ``include/fedavg_hip.h`` (FEDAVG_QSGD_F32: a 16-byte header (norm, level), the
slots, the packed sign bits; FEDAVG_NNADQ_F32: a 32-byte header (lo, step, levels), the codes).
``FedAVGAlgorithm`` passes record pointers to the kernels with the record's input format and
the kernel folds ``round(f64(x_hat) * w)`` per element with x_hat computed in the codec's
dtype — the same value the host dequantisation would have produced — while reading about 1
byte per element instead of 4 or 8:

* QSGD: x_hat = ((norm * sign) * slot) / level;
* NNADQ: x_hat = code * step + lo.

Both codecs live in the unvendored ``cyy_torch_algorithm`` (git ``@main``, quantization.
stochastic / quantization.deterministic); they are restated here (QSGD from the published
scheme; NNADQ as a deterministic adaptive-level affine code), so parity with that package is
unpinned (``oracle/qsgd_oracle.py`` and ``oracle/nnadq_oracle.py`` say what exactly is claimed).
``stochastic_quantization`` and ``NNADQ`` below are this framework's client-side quantisers (and
host dequantisers for consumers that need dense tensors, e.g. workers receiving a quantised
broadcast); the server-side hot path never calls ``dequantize_tensor``.
"""

from __future__ import annotations

import logging
import math
from collections.abc import Callable, Mapping
from dataclasses import dataclass

import torch

from . import _native
from .fedavg import ModelLayout

_log = logging.getLogger(__name__)

HEADER_BYTES = 16  # QSGD records
NNADQ_HEADER_BYTES = 32
DEFAULT_LEVEL = 255  # quantized_endpoint.py:104,110
NNADQ_MAX_LEVELS = 255  # one byte per code


def _align16(n: int) -> int:
    return (n + 15) // 16 * 16


@dataclass(frozen=True)
class QuantizedDtype:
    """Input format code of quantised records for the C ABI (``fedavg_dtype``)."""

    name: str
    value_dtype: torch.dtype  # the codec's arithmetic dtype (what dequant returns)
    code: int
    scheme: str = "qsgd"  # "qsgd" | "nnadq"

    def record_bytes(self, numel: int) -> int:
        """Byte size of one record of a numel-element tensor (== fedavg_<scheme>_record_bytes)."""
        if self.scheme == "nnadq":
            return NNADQ_HEADER_BYTES + _align16(numel)
        return record_bytes(numel)


QSGD_F32 = QuantizedDtype("qsgd_f32", torch.float32, _native.QSGD_F32)
QSGD_F64 = QuantizedDtype("qsgd_f64", torch.float64, _native.QSGD_F64)
NNADQ_F32 = QuantizedDtype("nnadq_f32", torch.float32, _native.NNADQ_F32, "nnadq")
NNADQ_F64 = QuantizedDtype("nnadq_f64", torch.float64, _native.NNADQ_F64, "nnadq")


def codec_for(dtype: torch.dtype, scheme: str = "qsgd") -> QuantizedDtype:
    if scheme == "nnadq":
        return NNADQ_F64 if dtype == torch.float64 else NNADQ_F32
    return QSGD_F64 if dtype == torch.float64 else QSGD_F32


def sign_offset(numel: int) -> int:
    """Byte offset of the sign bits in a record (== fedavg_qsgd_sign_offset)."""
    return HEADER_BYTES + _align16(numel)


def record_bytes(numel: int) -> int:
    """Byte size of one record (== fedavg_qsgd_record_bytes)."""
    return sign_offset(numel) + _align16((numel + 7) // 8)


@dataclass
class QuantizedTensor:
    """One quantised parameter tensor: a record (uint8, 1-D) + its shape and codec."""

    record: torch.Tensor
    shape: tuple[int, ...]
    codec: QuantizedDtype

    def __post_init__(self) -> None:
        self.shape = tuple(int(s) for s in self.shape)
        if self.record.dtype != torch.uint8 or self.record.dim() != 1:
            raise ValueError("a quantised record is a 1-D uint8 tensor")
        need = self.codec.record_bytes(self.numel)
        if self.record.numel() != need:
            raise ValueError(f"record holds {self.record.numel()} bytes, the layout needs {need}")

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

    def _qsgd(self) -> None:
        if self.codec.scheme != "qsgd":
            raise AttributeError(f"{self.codec.name} records have no QSGD fields")

    def _nnadq(self) -> None:
        if self.codec.scheme != "nnadq":
            raise AttributeError(f"{self.codec.name} records have no NNADQ fields")

    @property
    def norm(self) -> float:
        self._qsgd()
        return float(self.record[0:8].cpu().view(torch.float64)[0])

    @property
    def level(self) -> int:
        self._qsgd()
        return int(self.record[8:12].cpu().view(torch.int32)[0])

    @property
    def slots(self) -> torch.Tensor:
        self._qsgd()
        return self.record[HEADER_BYTES : HEADER_BYTES + self.numel]

    @property
    def sign_bits(self) -> torch.Tensor:
        """One 0/1 (uint8) per element, 1 = non-negative."""
        self._qsgd()
        so = sign_offset(self.numel)
        packed = self.record[so : so + (self.numel + 7) // 8]
        shifts = torch.arange(7, -1, -1, device=packed.device, dtype=torch.uint8)
        return ((packed.unsqueeze(1) >> shifts) & 1).reshape(-1)[: self.numel]

    @property
    def lo(self) -> float:
        self._nnadq()
        return float(self.record[0:8].cpu().view(torch.float64)[0])

    @property
    def step(self) -> float:
        self._nnadq()
        return float(self.record[8:16].cpu().view(torch.float64)[0])

    @property
    def levels(self) -> int:
        self._nnadq()
        return int(self.record[16:20].cpu().view(torch.int32)[0])

    @property
    def codes(self) -> torch.Tensor:
        self._nnadq()
        return self.record[NNADQ_HEADER_BYTES : NNADQ_HEADER_BYTES + self.numel]

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
    """Dense x_hat in the codec's dtype (host-side consumers; the server's FedAvg fold
    dequantises inside the kernel instead): QSGD ((norm * sign) * slot) / level, NNADQ
    code * step + lo."""
    dt = q.codec.value_dtype
    rec = q.record
    if q.codec.scheme == "nnadq":
        lo = rec[0:8].view(torch.float64).to(dt)
        step = rec[8:16].view(torch.float64).to(dt)
        return (q.codes.to(dt) * step + lo).reshape(q.shape)  # two eager ops: two roundings
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


def record_layout(numels: list[int], codec: QuantizedDtype = QSGD_F32) -> ModelLayout:
    """Byte layout of one client's records in one bucket (every record 16-B aligned)."""
    return ModelLayout(names=tuple(f"r{i}" for i in range(len(numels))),
                       shapes=tuple((codec.record_bytes(n),) for n in numels))


# -- NNADQ (NNADQClientEndpoint / NNADQServerEndpoint, quantized_endpoint.py:114-142) ----------

def nnadq_levels(lo: float, hi: float, weight: float) -> int:
    """Levels of one tensor's code: the step is at most ``weight`` x the tensor's largest
    magnitude, capped at 255 levels (one byte per code); 1 for a constant or non-finite tensor."""
    amax = max(abs(lo), abs(hi))
    if not (amax > 0 and weight > 0):
        return 1
    r = (hi - lo) / (weight * amax)
    if not math.isfinite(r) or r <= 0:
        return 1
    return int(min(NNADQ_MAX_LEVELS, max(1, math.ceil(r))))


def nnadq_quantize_tensor(tensor: torch.Tensor, weight: float = 0.01) -> QuantizedTensor:
    """Deterministic NNADQ quantisation of one tensor (on its own device): lo = min, hi = max,
    L = nnadq_levels(lo, hi, weight), step = (hi - lo) / L, code = clamp(round((x - lo) / step),
    0, L) (round half to even), all in the codec's dtype."""
    codec = codec_for(tensor.dtype, "nnadq")
    dt = codec.value_dtype
    v = tensor.detach().reshape(-1).to(dt)
    n = v.numel()
    dev = v.device
    rec = torch.zeros(codec.record_bytes(n), dtype=torch.uint8, device=dev)
    levels = 1
    if n:
        lo, hi = v.min(), v.max()
        levels = nnadq_levels(float(lo), float(hi), weight)
        step = (hi - lo) / torch.tensor(levels, dtype=dt, device=dev)
        s = float(step)
        if s > 0 and math.isfinite(s):
            codes = torch.clamp(torch.round((v - lo) / step), 0, levels)
            codes = torch.nan_to_num(codes, nan=0.0).to(torch.uint8)
        else:
            codes = torch.zeros(n, dtype=torch.uint8, device=dev)
        rec[NNADQ_HEADER_BYTES : NNADQ_HEADER_BYTES + n] = codes
        rec[0:8] = lo.to(torch.float64).reshape(1).view(torch.uint8)
        rec[8:16] = step.to(torch.float64).reshape(1).view(torch.uint8)
    rec[16:20] = torch.tensor([levels], dtype=torch.int32).view(torch.uint8).to(dev)
    return QuantizedTensor(rec, tuple(tensor.shape), codec)


class NeuralNetworkAdaptiveDeterministicQuant:
    """The client-side NNADQ quantiser (``NNADQ(weight)[0]``): every tensor of a parameter dict
    to an NNADQ record."""

    def __init__(self, weight: float) -> None:
        self.weight = float(weight)

    def __call__(self, parameter: Mapping[str, torch.Tensor]) -> dict[str, QuantizedTensor]:
        return {k: nnadq_quantize_tensor(v, self.weight) for k, v in parameter.items()}

    @staticmethod
    def check_compression_ratio(quantized_data: object, prefix: str = "") -> float:
        """Bytes of the records over the bytes of the dense tensors they replace (the endpoint's
        ``_after_quant`` log, quantized_endpoint.py:121-124,139-142); returned, not asserted."""
        parameter = getattr(quantized_data, "parameter", quantized_data)
        packed = dense = 0
        for v in parameter.values():
            if isinstance(v, QuantizedTensor):
                packed += v.record.numel()
                dense += v.numel * torch.empty((), dtype=v.codec.value_dtype).element_size()
        ratio = packed / dense if dense else 1.0
        _log.debug("%s compression ratio %.4f", prefix, ratio)
        return ratio


class NeuralNetworkAdaptiveDeterministicDequant:
    """The server-side NNADQ dequantiser (``NNADQServerEndpoint(weight=None)``'s dequant,
    quantized_endpoint.py:130-133): needs nothing but the records. The fused FedAvg path never
    calls it; dense consumers do."""

    def __call__(self, parameter: Mapping[str, object]) -> dict[str, object]:
        return dequantize_parameter(parameter)


def NNADQ(weight: float) -> tuple[NeuralNetworkAdaptiveDeterministicQuant, NeuralNetworkAdaptiveDeterministicDequant]:  # noqa: N802
    """The (quant, dequant) pair the NNADQ endpoints take (quantized_endpoint.py:117,135)."""
    return NeuralNetworkAdaptiveDeterministicQuant(weight), NeuralNetworkAdaptiveDeterministicDequant()
