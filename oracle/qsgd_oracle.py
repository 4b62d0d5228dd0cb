"""ORACLE — test infrastructure only, never product code.

CPU restatement (numpy) of the server-side dequantisation that the reference applies to every
quantised client update before FedAvg folds it:

  * ``QuantServerEndpoint.get`` — simulation_lib/topology/quantized_endpoint.py:69-77:
    ``data.parameter = self._dequant(data.parameter)`` (``delta_parameter`` for deltas);
  * ``StochasticQuantServerEndpoint`` — quantized_endpoint.py:102-111:
    ``quant, dequant = stochastic_quantization(quantization_level=255)``;
  * the dense result then goes through ``FedAVGAlgorithm`` (fed_avg_algorithm.py:43-99),
    restated and pinned in ``fedavg_oracle.py``.

PARITY UNPINNED. The codec itself lives in the third-party package ``cyy_torch_algorithm``
(``cyy_torch_algorithm.quantization.stochastic.stochastic_quantization``), which the reference
pins only as ``git+https://github.com/cyyever/torch_algorithm.git@main`` (pyproject.toml:12,
no revision). It is not vendored under /root/reference and not installed here, and the
reference holds no test, fixture or golden vector for it. What is restated below is the
published QSGD scheme (Alistarh et al., "QSGD: Communication-Efficient SGD via Gradient
Quantization and Encoding", NeurIPS 2017) in the form the reference's call sites use — one
norm per tensor, ``quantization_level`` = s = 255 so a slot fits a uint8, signs as packed bits:

  quant(x):   n = max|x| (the inf-norm; l2 when use_l2_norm), r = |x| / n * s,
              slot = floor(r) + Bernoulli(r - floor(r)), sign bit = not (x < 0)
  dequant:    x_hat = n * sign * slot / s, evaluated left to right in the codec's dtype

The bit-exact claim of the HIP kernel is therefore "identical to THIS dequantisation followed by
the pinned FedAvg fold", not "identical to cyy_torch_algorithm". The record byte layout is this
framework's own wire format (include/fedavg_hip.h, FEDAVG_QSGD_F32).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.
"""

from __future__ import annotations

import numpy as np

LEVEL = 255
HEADER_BYTES = 16


def _align16(n: int) -> int:
    return (n + 15) // 16 * 16


def sign_offset(numel: int) -> int:
    return HEADER_BYTES + _align16(numel)


def record_bytes(numel: int) -> int:
    return sign_offset(numel) + _align16((numel + 7) // 8)


def make_record(norm: float, level: int, slots: np.ndarray, sign_bits: np.ndarray) -> np.ndarray:
    """Assemble one record (uint8) from its fields; sign_bits is one 0/1 per element."""
    n = slots.size
    rec = np.zeros(record_bytes(n), dtype=np.uint8)
    rec[0:8] = np.frombuffer(np.float64(norm).tobytes(), dtype=np.uint8)
    rec[8:12] = np.frombuffer(np.int32(level).tobytes(), dtype=np.uint8)
    rec[HEADER_BYTES : HEADER_BYTES + n] = slots.astype(np.uint8)
    packed = np.packbits(sign_bits.astype(np.uint8))  # big-endian bit order, zero padded
    so = sign_offset(n)
    rec[so : so + packed.size] = packed
    return rec


def quantize(x: np.ndarray, rng: np.random.Generator, level: int = LEVEL, use_l2_norm: bool = False) -> np.ndarray:
    """QSGD quantisation of one tensor into a record (the client side; inputs for the tests).

    The codec dtype is float64 for float64 tensors and float32 otherwise; the norm is stored
    as that dtype's value widened to fp64. An all-zero tensor (norm 0) gets slot 0 everywhere.
    """
    dt = np.float64 if x.dtype == np.float64 else np.float32
    v = np.asarray(x, dtype=dt).reshape(-1)
    with np.errstate(invalid="ignore"):
        norm = dt(np.sqrt(np.sum(v.astype(np.float64) ** 2))) if use_l2_norm else dt(np.max(np.abs(v)) if v.size else 0)
        if norm > 0:
            r = (np.abs(v) / norm) * dt(level)
            fl = np.floor(r)
            slots = fl + (rng.random(v.size) < (r - fl))
        else:
            slots = np.zeros(v.size)
    slots = np.clip(slots, 0, level).astype(np.uint8)
    sign_bits = ~(v < 0)
    return make_record(float(norm), level, slots, sign_bits)


def parse(record: np.ndarray, numel: int) -> tuple[float, int, np.ndarray, np.ndarray]:
    """(norm, level, slots uint8[numel], sign bits uint8[numel]) of one record."""
    rec = np.asarray(record, dtype=np.uint8)
    norm = float(rec[0:8].view(np.float64)[0])
    level = int(rec[8:12].view(np.int32)[0])
    slots = rec[HEADER_BYTES : HEADER_BYTES + numel].copy()
    so = sign_offset(numel)
    bits = np.unpackbits(rec[so : so + (numel + 7) // 8])[:numel]
    return norm, level, slots, bits


def dequantize(record: np.ndarray, numel: int, codec_dtype) -> np.ndarray:
    """x_hat = ((norm * sign) * slot) / level, each operation rounded in the codec's dtype
    (numpy float32 / float64 array ops round per operation and never fuse)."""
    dt = np.dtype(codec_dtype).type
    norm, level, slots, bits = parse(record, numel)
    sign = np.where(bits.astype(bool), dt(1), dt(-1))
    with np.errstate(invalid="ignore", over="ignore"):
        return ((dt(norm) * sign) * slots.astype(dt)) / dt(level)
