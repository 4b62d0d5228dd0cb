"""Generate the golden PersonalizedFedAVG fixtures from the REFERENCE's own code.

Runs only in the build container (the reference is mounted read-only at /root/reference); a
no-op elsewhere. It loads, unmodified, the reference's
  simulation_lib/message.py, simulation_lib/algorithm/aggregation_algorithm.py,
  simulation_lib/algorithm/fed_avg_algorithm.py,
  simulation_lib/algorithm/personalized_aggregation_algorithm.py
through the same arithmetic-free stubs as gen_golden.py (see its header), and drives
``PersonalizedFedAVGAlgorithm`` exactly like the server does: ``set_worker_weights`` once, one
``process_worker_data`` per arrival (None = a skipped worker), then ``aggregate_worker_data``.

Output: tests/golden/personalized_golden.npz (inputs, per-receiver outputs, centralized output)
and tests/golden/personalized_manifest.json. Re-run: `python tests/golden/gen_personalized.py`.
"""

from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

from gen_golden import REF, _ds_weights, _load_reference, _model, _np  # noqa: E402


def build_cases():
    """Each case: dict(name, shapes, dtype, worker_weights {recv: {client: w}},
    arrivals=[(wid, params|None, other)])."""
    cases = []

    def add(name, shapes, dtype, workers, worker_weights, seed, order=None):
        order = list(range(workers)) if order is None else order
        arrivals = [(k, _model(shapes, dtype, seed + k), {}) for k in order]
        c = dict(name=name, shapes=shapes, dtype=dtype, worker_weights=worker_weights,
                 arrivals=arrivals, expect_error=None)
        cases.append(c)
        return c

    def dense(n, seed, lo=0.05, hi=3.0):
        rng = np.random.default_rng(seed)
        return {j: {i: float(rng.uniform(lo, hi)) for i in range(n) if i != j} for j in range(n)}

    # float similarity weights (inexact products: the separately rounded mul + add path)
    add("p_n4_f32", {"a": (7,), "b": (3, 5), "c": (33, 17)}, torch.float32, 4, dense(4, 1), 1)
    # integer weights (exact products: the fused fold); missing entries default to 0 (:36)
    rng = np.random.default_rng(2)
    ww = {j: {i: int(rng.integers(1, 500)) for i in range(6) if i != j and (i + j) % 4 != 1} for j in range(6)}
    add("p_n6_int_sparse", {"w": (2049,), "x": (5, 7, 9), "s": ()}, torch.float32, 6, ww, 2)
    add("p_n16_f32", {"conv": (16, 3, 3, 3), "bn": (16,), "fc": (10, 64), "big": (3001,)}, torch.float32,
        16, dense(16, 3), 3)
    add("p_n3_f16", {"h0": (1500,), "h1": (8, 9)}, torch.float16, 3, dense(3, 4), 4)
    add("p_n3_bf16", {"b0": (1500,), "b1": (8, 9)}, torch.bfloat16, 3, dense(3, 5), 5)
    add("p_n3_f64", {"d0": (2051,), "d1": (3,)}, torch.float64, 3, dense(3, 6), 6)
    # arrivals out of worker-id order; receivers listed in a non-sorted key order (the
    # centralized average folds in key order, personalized_aggregation_algorithm.py:51-53)
    w5 = dense(5, 7)
    add("p_order", {"r0": (2500,), "r1": (40,)}, torch.float32, 5,
        {j: w5[j] for j in (3, 0, 4, 1, 2)}, 7, order=[2, 4, 0, 3, 1])
    # receivers are a subset of the senders: clients 3 and 4 feed every receiver
    rng = np.random.default_rng(8)
    add("p_subset", {"u": (777,)}, torch.float32, 5,
        {j: {i: float(rng.uniform(0.1, 2.0)) for i in range(5) if i != j} for j in (0, 1, 2)}, 8)
    # a skipped worker (None) contributes to nobody
    c = add("p_skipped", {"s0": (1031,), "s1": (17,)}, torch.float32, 5, dense(5, 9), 9)
    c["arrivals"][2] = (2, None, {})
    # signed zeros through the first fold (an assignment in the reference)
    c = add("p_signed_zero", {"z": (64,)}, torch.float32, 3, {0: {1: 2.0, 2: 3.0}, 1: {0: 1.0, 2: 1.0},
                                                             2: {0: 0.5, 1: 4.0}}, 10)
    for a in c["arrivals"]:
        a[1]["z"][:] = -0.0
    # the largest receiver block of the kernel (64 receivers) and beyond it (80: two blocks)
    add("p_n64", {"q0": (300,), "q1": (65,)}, torch.float32, 64, dense(64, 11), 11)
    add("p_n80", {"q0": (200,), "q1": (3,)}, torch.float32, 80, dense(80, 12), 12)
    # dataset-size-like integer weights on every pair
    rng = np.random.default_rng(13)
    add("p_n8_ds", {"k0": (4099,)}, torch.float32, 8,
        {j: {i: int(rng.integers(100, 5001)) for i in range(8) if i != j} for j in range(8)}, 13)
    # other_data agreed by every client is passed through per receiver
    c = add("p_other_data", {"o": (100,)}, torch.float32, 3, dense(3, 14), 14)
    for a in c["arrivals"]:
        a[2]["round"] = 5

    # ---- errors ----
    c = add("p_err_nan_input", {"e": (100,)}, torch.float32, 3, dense(3, 20), 20)
    c["arrivals"][1][1]["e"][17] = float("nan")
    c["expect_error"] = "AssertionError"
    # receiver 0 only has zero weights: 0 / 0 (fed_avg_algorithm.py:97)
    c = add("p_err_zero_total", {"e": (100,)}, torch.float32, 3, {0: {}, 1: {0: 1.0, 2: 1.0}, 2: {0: 1, 1: 1}}, 21)
    c["expect_error"] = "AssertionError"
    # receiver 1 hears from nobody: its FedAVG has nothing accumulated (fed_avg_algorithm.py:88)
    c = add("p_err_no_data", {"e": (100,)}, torch.float32, 2, {0: {1: 1.0}, 1: {0: 1.0}}, 22)
    c["arrivals"] = [c["arrivals"][1]]
    c["expect_error"] = "AssertionError"
    c = add("p_err_other_data", {"e": (100,)}, torch.float32, 3, dense(3, 23), 23)
    c["arrivals"][0][2]["round"] = 1
    c["arrivals"][1][2]["round"] = 2
    c["expect_error"] = "RuntimeError"
    # inf with a zero weight: inf * 0 = NaN in the receiver that weighs it 0 (:54, :93)
    c = add("p_err_inf_zero_weight", {"e": (100,)}, torch.float32, 3,
            {0: {1: 1.0, 2: 0.0}, 1: {0: 1.0, 2: 1.0}, 2: {0: 1.0, 1: 1.0}}, 24)
    c["arrivals"][2][1]["e"][3] = float("inf")
    c["expect_error"] = "AssertionError"
    return cases


def run_reference(case, message, pers):
    algo = pers.PersonalizedFedAVGAlgorithm()
    algo.set_worker_weights({j: dict(v) for j, v in case["worker_weights"].items()})
    for wid, params, other in case["arrivals"]:
        msg = None
        if params is not None:
            msg = message.ParameterMessage(parameter={k: v.clone() for k, v in params.items()},
                                           other_data=dict(other))
        algo.process_worker_data(worker_id=wid, worker_data=msg)
    return algo.aggregate_worker_data()


def main() -> int:
    if not REF.exists():
        print("reference not present: nothing to generate")
        return 0
    message, _agg, _fed = _load_reference()
    pers = importlib.import_module("simulation_lib.algorithm.personalized_aggregation_algorithm")
    arrays: dict[str, np.ndarray] = {}
    manifest = {"generator": "tests/golden/gen_personalized.py",
                "reference_files": ["simulation_lib/message.py",
                                    "simulation_lib/algorithm/aggregation_algorithm.py",
                                    "simulation_lib/algorithm/fed_avg_algorithm.py",
                                    "simulation_lib/algorithm/personalized_aggregation_algorithm.py"],
                "cases": []}
    for case in build_cases():
        name = case["name"]
        entry = {
            "name": name,
            "dtype": str(case["dtype"]).replace("torch.", ""),
            "names": list(case["shapes"].keys()),
            "shapes": [list(s) for s in case["shapes"].values()],
            # JSON keys are strings: keep the receiver order as a list of [recv, [[client, w], ...]]
            "worker_weights": [[j, [[i, w] for i, w in v.items()]] for j, v in case["worker_weights"].items()],
            "arrivals": [],
        }
        for n, (wid, params, other) in enumerate(case["arrivals"]):
            entry["arrivals"].append({"worker_id": wid, "other_data": other,
                                      "keys": None if params is None else list(params.keys())})
            if params is not None:
                for k, v in params.items():
                    arrays[f"{name}/in/{n}/{k}"] = _np(v)
        try:
            res = run_reference(case, message, pers)
        except (AssertionError, RuntimeError) as e:
            entry["error"] = type(e).__name__
            assert case["expect_error"] == entry["error"], (name, repr(e))
        else:
            assert case["expect_error"] is None, f"{name}: expected {case['expect_error']}"
            entry["error"] = None
            entry["receivers"] = []
            for j, msg in res.worker_data.items():
                entry["receivers"].append({"worker_id": j, "keys": list(msg.parameter.keys()),
                                           "other_data": msg.other_data, "in_round": msg.in_round,
                                           "end_training": msg.end_training})
                for k, v in msg.parameter.items():
                    assert v.dtype == torch.float64
                    arrays[f"{name}/out/{j}/{k}"] = v.numpy()
            central = res.other_data["centralized_parameter"]
            entry["central_keys"] = list(central.keys())
            for k, v in central.items():
                arrays[f"{name}/central/{k}"] = v.numpy()
        manifest["cases"].append(entry)
        print(f"{name}: {'error ' + entry['error'] if entry['error'] else 'ok'}")
    np.savez_compressed(HERE / "personalized_golden.npz", **arrays)
    (HERE / "personalized_manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")
    size = (HERE / "personalized_golden.npz").stat().st_size
    print(f"wrote {len(manifest['cases'])} cases, {size / 1e6:.2f} MB")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
