"""ORACLE — test infrastructure only, never product code.

CPU restatement (numpy) of the server-side dequantisation behind ``NNADQServerEndpoint``:

  * ``QuantServerEndpoint.get`` — simulation_lib/topology/quantized_endpoint.py:69-77:
    ``data.parameter = self._dequant(data.parameter)`` (``delta_parameter`` for deltas);
  * ``NNADQClientEndpoint`` / ``NNADQServerEndpoint`` — quantized_endpoint.py:114-142:
    ``quant, dequant = NNADQ(weight=weight)`` on the workers, and on the server either the same
    pair or a bare ``NeuralNetworkAdaptiveDeterministicDequant()`` (weight None, :130-133);
  * the dense result then goes through ``FedAVGAlgorithm`` (fed_avg_algorithm.py:43-99),
    restated and pinned in ``fedavg_oracle.py``.

PARITY UNPINNED. The codec lives in the third-party package ``cyy_torch_algorithm``
(``cyy_torch_algorithm.quantization.deterministic``), pinned by the reference only as
``git+https://github.com/cyyever/torch_algorithm.git@main`` (pyproject.toml:12, no revision);
it is not vendored under /root/reference, not installed here, and the reference holds no test,
fixture or golden vector for it. What is restated is a deterministic per-tensor affine
(min / step) quantiser whose number of levels adapts to each tensor through ``weight`` — the
shape the endpoint's call sites imply (a ``weight`` knob on the client, a stateless server
dequantiser that needs nothing but the payload) — with this framework's own record layout
(include/fedavg_hip.h, FEDAVG_NNADQ_F32):

  quant(x, weight):  lo = min(x), hi = max(x)                       (codec dtype)
                     L  = clamp(ceil((hi - lo) / (weight * max(|lo|, |hi|))), 1, 255)
                          (fp64; L = 1 when that is not a finite positive number)
                     step = (hi - lo) / L                            (codec dtype)
                     code = clamp(rint((x - lo) / step), 0, L)       (0 when step == 0)
  dequant:           x_hat = code * step + lo, two roundings in the codec's dtype

The codec dtype is float64 for float64 tensors and float32 otherwise. NaN in a tensor makes
lo / hi NaN, and every dequantised element NaN (the server's NaN check then fires, as it would
on the dense tensor). The bit-exact claim of the HIP kernel is "identical to THIS dequantisation
followed by the pinned FedAvg fold", not "identical to cyy_torch_algorithm".

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.
"""

from __future__ import annotations

import math

import numpy as np

HEADER_BYTES = 32
MAX_LEVELS = 255


def _align16(n: int) -> int:
    return (n + 15) // 16 * 16


def record_bytes(numel: int) -> int:
    return HEADER_BYTES + _align16(numel)


def choose_levels(lo: float, hi: float, weight: float) -> int:
    """Number of levels L (codes 0..L) for one tensor: the step is at most weight x the
    tensor's largest magnitude, capped at 255 levels (one byte per code)."""
    amax = max(abs(lo), abs(hi))
    with np.errstate(all="ignore"):
        r = (hi - lo) / (weight * amax) if amax > 0 and weight > 0 else float("nan")
    if not math.isfinite(r) or r <= 0:
        return 1
    return int(min(MAX_LEVELS, max(1, math.ceil(r))))


def make_record(lo: float, step: float, levels: int, codes: np.ndarray) -> np.ndarray:
    n = codes.size
    rec = np.zeros(record_bytes(n), dtype=np.uint8)
    rec[0:8] = np.frombuffer(np.float64(lo).tobytes(), dtype=np.uint8)
    rec[8:16] = np.frombuffer(np.float64(step).tobytes(), dtype=np.uint8)
    rec[16:20] = np.frombuffer(np.int32(levels).tobytes(), dtype=np.uint8)
    rec[HEADER_BYTES : HEADER_BYTES + n] = codes.astype(np.uint8)
    return rec


def quantize(x: np.ndarray, weight: float = 0.01) -> np.ndarray:
    """Deterministic quantisation of one tensor into a record (client side; test inputs)."""
    dt = np.float64 if x.dtype == np.float64 else np.float32
    v = np.asarray(x, dtype=dt).reshape(-1)
    if v.size == 0:
        return make_record(0.0, 0.0, 1, np.zeros(0, dtype=np.uint8))
    lo, hi = dt(np.min(v)), dt(np.max(v))
    levels = choose_levels(float(lo), float(hi), weight)
    with np.errstate(all="ignore"):
        step = dt(hi - lo) / dt(levels)
        if step > 0 and np.isfinite(step):
            codes = np.clip(np.rint((v - lo) / step), 0, levels)
        else:
            codes = np.zeros(v.size)
    codes = np.nan_to_num(codes, nan=0.0).astype(np.uint8)
    return make_record(float(lo), float(step), levels, codes)


def parse(record: np.ndarray, numel: int) -> tuple[float, float, int, np.ndarray]:
    """(lo, step, levels, codes uint8[numel]) of one record."""
    rec = np.asarray(record, dtype=np.uint8)
    lo = float(rec[0:8].view(np.float64)[0])
    step = float(rec[8:16].view(np.float64)[0])
    levels = int(rec[16:20].view(np.int32)[0])
    return lo, step, levels, rec[HEADER_BYTES : HEADER_BYTES + numel].copy()


def dequantize(record: np.ndarray, numel: int, codec_dtype) -> np.ndarray:
    """x_hat = code * step + lo, each operation rounded in the codec's dtype (numpy array ops
    round per operation and never fuse)."""
    dt = np.dtype(codec_dtype).type
    lo, step, _, codes = parse(record, numel)
    with np.errstate(invalid="ignore", over="ignore"):
        return codes.astype(dt) * dt(step) + dt(lo)
