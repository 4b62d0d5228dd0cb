"""Readers for the golden fixtures generated from the reference (tests/golden/gen_golden.py)."""

from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Any

import numpy as np
import torch

GOLDEN_DIR = Path(__file__).resolve().parent / "golden"


@dataclass
class Arrival:
    worker_id: int
    weight: Any
    other_data: dict
    arrays: dict[str, np.ndarray] | None  # raw (bf16 as uint16 bits)
    elem_weights: dict[str, np.ndarray] | None = None  # per-element _get_weight values (weight_mode)


@dataclass
class GoldenCase:
    name: str
    dtype: str
    names: list[str]
    shapes: list[tuple[int, ...]]
    accumulate: bool
    aggregate_loss: bool
    per_tensor_weight: dict | None
    arrivals: list[Arrival]
    error: str | None
    expected: dict[str, np.ndarray] | None
    meta: dict
    kinds: list[str] | None = None  # per arrival "full" / "delta" (delta: against `old`)
    old: dict[str, np.ndarray] | None = None
    # overridden hooks (gen_golden.make_hooked_class): None, "scalar_tensor_float32/64",
    # "elementwise_float32/64"; total_weight_hook: None or "scaled" ((x * 3) / (W + 1))
    weight_mode: str | None = None
    total_weight_hook: str | None = None

    def torch_params(self, arrival: Arrival, device: torch.device | str = "cpu") -> dict[str, torch.Tensor]:
        assert arrival.arrays is not None
        out = {}
        for k, a in arrival.arrays.items():
            if self.dtype == "bfloat16":
                t = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
            else:
                t = torch.from_numpy(a.copy())
            out[k] = t.to(device)
        return out


def load_golden() -> dict[str, GoldenCase]:
    manifest = json.loads((GOLDEN_DIR / "manifest.json").read_text())
    data = np.load(GOLDEN_DIR / "fedavg_golden.npz", allow_pickle=False)
    cases = {}
    for c in manifest["cases"]:
        name = c["name"]
        arrivals = []
        for j, a in enumerate(c["arrivals"]):
            arrays = None
            if a["keys"] is not None:
                arrays = {k: data[f"{name}/in/{j}/{k}"] for k in a["keys"]}
            ew = None
            if (c.get("weight_mode") or "").startswith("elementwise") and a["keys"] is not None:
                ew = {k: data[f"{name}/w/{j}/{k}"] for k in c["names"]}
            arrivals.append(Arrival(a["worker_id"], a["weight"], dict(a["other_data"]), arrays, ew))
        expected = None
        if c["error"] is None:
            expected = {k: data[f"{name}/out/{k}"] for k in c["out_keys"]}
        cases[name] = GoldenCase(
            name=name,
            dtype=c["dtype"],
            names=c["names"],
            shapes=[tuple(s) for s in c["shapes"]],
            accumulate=c["accumulate"],
            aggregate_loss=c["aggregate_loss"],
            per_tensor_weight=c["per_tensor_weight"],
            arrivals=arrivals,
            error=c["error"],
            expected=expected,
            meta=c,
            kinds=c.get("kinds"),
            old={k: data[f"{name}/old/{k}"] for k in c["old_keys"]} if c.get("old_keys") else None,
            weight_mode=c.get("weight_mode"),
            total_weight_hook=c.get("total_weight_hook"),
        )
    return cases


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    """Bit-for-bit equality of float64 arrays (distinguishes -0.0 / +0.0, NaN payloads)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


# ---- PersonalizedFedAVG fixtures (tests/golden/gen_personalized.py) ----------------------
@dataclass
class PersonalizedCase:
    name: str
    dtype: str
    names: list[str]
    shapes: list[tuple[int, ...]]
    worker_weights: dict[int, dict[int, Any]]  # receiver -> {client: weight}, key order kept
    arrivals: list[Arrival]  # Arrival.weight is unused (None)
    error: str | None
    expected: dict[int, dict[str, np.ndarray]] | None  # receiver -> {name: fp64}
    central: dict[str, np.ndarray] | None
    meta: dict

    def torch_params(self, arrival: Arrival, device: torch.device | str = "cpu") -> dict[str, torch.Tensor]:
        return GoldenCase.torch_params(self, arrival, device)  # type: ignore[arg-type]


def load_personalized() -> dict[str, PersonalizedCase]:
    manifest = json.loads((GOLDEN_DIR / "personalized_manifest.json").read_text())
    data = np.load(GOLDEN_DIR / "personalized_golden.npz", allow_pickle=False)
    cases = {}
    for c in manifest["cases"]:
        name = c["name"]
        arrivals = []
        for n, a in enumerate(c["arrivals"]):
            arrays = None if a["keys"] is None else {k: data[f"{name}/in/{n}/{k}"] for k in a["keys"]}
            arrivals.append(Arrival(a["worker_id"], None, dict(a["other_data"]), arrays))
        expected = central = None
        if c["error"] is None:
            expected = {r["worker_id"]: {k: data[f"{name}/out/{r['worker_id']}/{k}"] for k in r["keys"]}
                        for r in c["receivers"]}
            central = {k: data[f"{name}/central/{k}"] for k in c["central_keys"]}
        cases[name] = PersonalizedCase(
            name=name, dtype=c["dtype"], names=c["names"], shapes=[tuple(s) for s in c["shapes"]],
            worker_weights={j: {i: w for i, w in row} for j, row in c["worker_weights"]},
            arrivals=arrivals, error=c["error"], expected=expected, central=central, meta=c,
        )
    return cases
