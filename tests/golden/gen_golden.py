"""Generate the golden FedAvg fixtures from the REFERENCE's own hot-path code.

Runs only in the build container, where the reference is mounted read-only at
/root/reference; it is a no-op elsewhere (the reference never travels to the GPU box).

What is imported: exactly three reference files, unmodified —
  simulation_lib/message.py, simulation_lib/algorithm/aggregation_algorithm.py,
  simulation_lib/algorithm/fed_avg_algorithm.py.
The rest of the reference's package (and its unvendored `cyy_*` dependencies, which are
not installed) is bypassed with stubs that carry no arithmetic:
  * typing.override  <- typing_extensions.override (the reference targets Python 3.12)
  * cyy_naive_lib.log                   -> logging shims (log_debug/log_info/log_error)
  * cyy_torch_toolbox.ModelParameter    -> dict (the reference's own type alias)
  * cyy_preprocessing_pipeline.tensor   -> recursive_tensor_op (only get_message_size uses it)
  * simulation_lib.config               -> DistributedTrainingConfig = object (type hint only)
  * simulation_lib, simulation_lib.algorithm -> namespace packages pointing at the reference
    directories, so their heavy __init__ files (process pools, trainers) are not executed.
All arithmetic on the path is the reference's torch code.

Output: tests/golden/fedavg_golden.npz (inputs + expected outputs) and
tests/golden/manifest.json (case metadata). Re-run: `python tests/golden/gen_golden.py`.
"""

from __future__ import annotations

import importlib
import json
import logging
import sys
import types
import typing
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT_DIR = Path(__file__).resolve().parent
sys.path.insert(0, str(OUT_DIR.parent.parent))  # the repo root: tests.golden_hooks
from tests.golden_hooks import make_hooked_class  # noqa: E402  (the cases' overridden hooks)


def _load_reference():
    import typing_extensions

    if not hasattr(typing, "override"):
        typing.override = typing_extensions.override  # type: ignore[attr-defined]

    def stub(name: str, **attrs):
        mod = types.ModuleType(name)
        mod.__dict__.update(attrs)
        sys.modules[name] = mod
        return mod

    log = logging.getLogger("reference")
    stub("cyy_naive_lib")
    stub("cyy_naive_lib.log", log_debug=log.debug, log_info=log.info, log_error=log.error,
         log_warning=log.warning)
    stub("cyy_torch_toolbox", ModelParameter=dict)
    stub("cyy_preprocessing_pipeline")
    stub("cyy_preprocessing_pipeline.tensor", recursive_tensor_op=lambda obj, fun: obj)
    pkg = stub("simulation_lib")
    pkg.__path__ = [str(REF / "simulation_lib")]
    alg = stub("simulation_lib.algorithm")
    alg.__path__ = [str(REF / "simulation_lib" / "algorithm")]
    stub("simulation_lib.config", DistributedTrainingConfig=object)
    message = importlib.import_module("simulation_lib.message")
    agg = importlib.import_module("simulation_lib.algorithm.aggregation_algorithm")
    fed = importlib.import_module("simulation_lib.algorithm.fed_avg_algorithm")
    return message, agg, fed


# --------------------------------------------------------------------------------------
# case definitions (inputs are torch tensors so that bf16/f16 are exact)
# --------------------------------------------------------------------------------------
def _gen(shape, dtype, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g, dtype=torch.float32) * scale).to(dtype)


def _model(shapes: dict[str, tuple[int, ...]], dtype, seed, scale=1.0):
    return {n: _gen(s, dtype, seed * 131 + i, scale) for i, (n, s) in enumerate(shapes.items())}


def _ds_weights(n, seed):
    rng = np.random.default_rng(seed)
    return [int(x) for x in rng.integers(100, 5001, size=n)]


SMALL_RESNET = {
    "conv1.weight": (16, 3, 3, 3),
    "bn1.weight": (16,),
    "bn1.bias": (16,),
    "layer1.conv.weight": (16, 16, 3, 3),
    "fc.weight": (10, 64),
    "fc.bias": (10,),
    "big": (6001,),
}


def build_cases():
    """Each case: dict(name, layout, dtype, arrivals=[(wid, params|None, weight, other)],
    accumulate, aggregate_loss, per_tensor_weight)."""
    cases = []

    def add(name, shapes, dtype, n, weights, seed, **kw):
        arrivals = []
        for k in range(n):
            arrivals.append((k, _model(shapes, dtype, seed + k), weights[k], {}))
        cases.append(dict(name=name, shapes=shapes, dtype=dtype, arrivals=arrivals,
                          accumulate=kw.get("accumulate", True), aggregate_loss=False,
                          per_tensor_weight=None, expect_error=None, weight_mode=None,
                          total_weight_hook=None))
        return cases[-1]

    add("n1_f32", {"a": (7,), "b": (3, 5), "c": (33, 17)}, torch.float32, 1, [250], 1)
    add("n3_f32_int", {"w": (2049,), "x": (5, 7, 9), "s": (), "y": (4099,)}, torch.float32, 3,
        _ds_weights(3, 3), 3)
    add("n16_f32_float", SMALL_RESNET, torch.float32, 16,
        [float(x) for x in np.random.default_rng(16).uniform(0.1, 10.0, 16)], 16)
    add("n64_f32_uniform", {"p0": (2048,), "p1": (2052,)}, torch.float32, 64, [1.0] * 64, 64)
    add("n64_f32_ds", {"q0": (3000,), "q1": (1025,)}, torch.float32, 64, _ds_weights(64, 65), 65)
    add("n8_f16", {"h0": (1500,), "h1": (8, 9)}, torch.float16, 8, _ds_weights(8, 8), 8)
    add("n8_bf16", {"b0": (1500,), "b1": (8, 9)}, torch.bfloat16, 8, _ds_weights(8, 9), 9)
    add("n8_f64", {"d0": (2051,), "d1": (3,)}, torch.float64, 8, _ds_weights(8, 10), 10)
    c = add("n4_large", {"l0": (4096,)}, torch.float32, 4, [5000, 1, 4999, 2], 11)
    for i, a in enumerate(c["arrivals"]):
        a[1]["l0"] *= 1e30 if i % 2 == 0 else 1e-30
    c = add("n3_subnormal", {"t0": (1000,)}, torch.float32, 3, [3, 5, 7], 12)
    for a in c["arrivals"]:
        a[1]["t0"] *= 1e-40

    # skipped client (None) contributes nothing (aggregation_algorithm.py:98-100)
    c = add("skipped", {"s0": (1031,), "s1": (17,)}, torch.float32, 4, [1, 3, 2, 5], 20)
    c["arrivals"][1] = (1, None, None, {})

    # same clients, reversed arrival order
    c = add("order_fwd", {"r0": (2500,)}, torch.float32, 16, _ds_weights(16, 30), 30)
    rev = dict(c)
    rev = dict(name="order_rev", shapes=c["shapes"], dtype=c["dtype"], arrivals=list(reversed(c["arrivals"])),
               accumulate=True, aggregate_loss=False, per_tensor_weight=None, expect_error=None)
    cases.append(rev)

    # ratio path (accumulate=False, aggregation_algorithm.py:51-76)
    c = add("ratio_path", SMALL_RESNET, torch.float32, 8, _ds_weights(8, 40), 40)
    c["accumulate"] = False
    c = add("ratio_path_f16", {"h": (777,)}, torch.float16, 5, [1, 2, 3, 4, 5], 41)
    c["accumulate"] = False

    # signed zeros: first contribution is an assignment, not 0 + tmp
    c = add("signed_zero", {"z": (64,)}, torch.float32, 2, [2, 3], 50)
    c["arrivals"][0][1]["z"][:] = -0.0
    c["arrivals"][1][1]["z"][:] = -0.0
    c = add("signed_zero_single", {"z": (5,)}, torch.float32, 1, [7], 51)
    c["arrivals"][0][1]["z"][:] = -0.0

    # negative weight is accepted on the streaming path
    add("negative_weight", {"n": (300,)}, torch.float32, 3, [5, -2, 4], 52)

    # fractional weights whose products are not exact in fp64
    add("inexact_weights", {"f": (1999,)}, torch.float32, 5, [0.1, 0.7, 1 / 3, 2.2, 1e-3], 53)

    # per-(client, tensor) weights through an overridden _get_weight (fed_avg_algorithm.py:66-69)
    # (the message's aggregation_weight is the client's row index into these tables)
    c = add("per_tensor_weight", {"u": (513,), "v": (129,)}, torch.float32, 4, [0, 1, 2, 3], 54)
    c["per_tensor_weight"] = {"u": [3, 1, 4, 1], "v": [0.5, 9, 2, 6]}

    # missing key in one client -> per-name totals
    c = add("missing_key", {"m0": (600,), "m1": (40,)}, torch.float32, 3, [2, 3, 4], 55)
    del c["arrivals"][1][1]["m1"]

    # loss averaging (fed_avg_algorithm.py:115-134)
    c = add("aggregate_loss", {"g": (100,)}, torch.float32, 3, [10, 30, 60], 56)
    c["aggregate_loss"] = True
    for i, a in enumerate(c["arrivals"]):
        a[3]["training_loss"] = [0.5, 1.5, 2.5][i]
        a[3]["epoch"] = 3

    # delta updates restored against the cached global model (message.py:40-61), mixed with a
    # full update, exactly as AggregationServer feeds them (aggregation_server.py:121-129)
    c = add("delta_restore", {"d0": (3001,), "d1": (17, 9)}, torch.float64, 5, [120, 4000, 33, 950, 7], 57)
    g = torch.Generator().manual_seed(570)
    c["old"] = {"d0": torch.randn(3001, generator=g, dtype=torch.float64),
                "d1": torch.randn(17, 9, generator=g, dtype=torch.float64)}
    c["kinds"] = ["delta", "delta", "full", "delta", "delta"]
    c["arrivals"][2] = (2, {k: v.to(torch.float32) for k, v in c["arrivals"][2][1].items()}, 33, {})

    # a key that first appears in a later client (fed_avg_algorithm.py:55-62 grow the per-name
    # dicts): output keys in first-seen order, per-name totals over the clients that sent it
    c = add("late_key", {"a": (300,), "b": (4099,), "c": (5, 3)}, torch.float32, 4, [7, 2, 9, 4], 58)
    del c["arrivals"][0][1]["b"], c["arrivals"][0][1]["c"]
    del c["arrivals"][1][1]["c"]
    del c["arrivals"][2][1]["a"]

    # _apply_total_weight overridden by a subclass (fed_avg_algorithm.py:71-74, used at :94-96);
    # the hook sees the per-name total and the fp64 weighted sum
    c = add("total_weight_hook", {"o0": (2050,), "o1": (6, 7)}, torch.float32, 5, _ds_weights(5, 59), 59)
    c["total_weight_hook"] = "scaled"

    # tensor-valued _get_weight (fed_avg_algorithm.py:51-54,66-69: `tmp = x.to(f64) * weight`,
    # `total += weight`): a fresh 0-dim tensor per (client, tensor) — the totals then accumulate in
    # the tensor's dtype — or a per-element weight tensor of the parameter's shape
    fw = [float(x) for x in np.random.default_rng(70).uniform(0.1, 10.0, 6)]
    c = add("weight_tensor_f32", {"s0": (1500,), "s1": (9,)}, torch.float32, 6, fw, 70)
    c["weight_mode"] = "scalar_tensor_float32"
    c = add("weight_tensor_f64", {"s0": (1500,), "s1": (9,)}, torch.float32, 6, fw, 71)
    c["weight_mode"] = "scalar_tensor_float64"
    for wdt, seed in (("float64", 72), ("float32", 73)):
        # (aggregation_weight is the arrival's row in elem_weights, as in per_tensor_weight)
        c = add(f"weight_elementwise_f{wdt[5:]}", {"e0": (2500,), "e1": (3, 11), "e2": ()}, torch.float32, 5,
                [0, 1, 2, 3, 4], seed)
        c["weight_mode"] = f"elementwise_{wdt}"
        g = torch.Generator().manual_seed(seed * 7)
        c["elem_weights"] = [
            {n: (torch.rand(sh, generator=g, dtype=torch.float64) * 4 + 0.25).to(getattr(torch, wdt))
             for n, sh in c["shapes"].items()}
            for _ in range(5)
        ]

    # a state dict of mixed dtypes (fp32 / fp16 / fp64 tensors, an int64 counter like
    # BatchNorm's num_batches_tracked, a 0-dim fp32 and an empty tensor): the reference converts
    # each tensor to fp64 on its own (`x.to(f64) * w`, fed_avg_algorithm.py:51-54)
    mixed = {"w": ((700,), torch.float32), "cnt": ((), torch.int64), "h": ((33,), torch.float16),
             "s": ((), torch.float32), "e": ((0,), torch.float32), "d": ((5, 2), torch.float64)}
    c = add("mixed_dtypes", {n: sh for n, (sh, _) in mixed.items()}, torch.float32, 4, _ds_weights(4, 74), 74)
    c["dtype"] = "mixed"
    for k, a in enumerate(c["arrivals"]):
        for i, (n, (sh, dt)) in enumerate(mixed.items()):
            if dt == torch.int64:
                a[1][n] = torch.tensor(1000 * (k + 1) + 7, dtype=torch.int64)
            else:
                a[1][n] = _gen(sh, dt, 74 * 131 + k * 17 + i)

    # ---- errors ----
    c = add("err_nan_input", {"e": (100,)}, torch.float32, 3, [1, 2, 3], 60)
    c["arrivals"][1][1]["e"][17] = float("nan")
    c["expect_error"] = "AssertionError"
    c = add("err_inf_minus_inf", {"e": (100,)}, torch.float32, 2, [1, 1], 61)
    c["arrivals"][0][1]["e"][5] = float("inf")
    c["arrivals"][1][1]["e"][5] = float("-inf")
    c["expect_error"] = "AssertionError"
    c = add("err_zero_total_weight", {"e": (100,)}, torch.float32, 2, [0, 0], 62)
    c["expect_error"] = "AssertionError"
    c = add("err_other_data_mismatch", {"e": (100,)}, torch.float32, 2, [1, 1], 63)
    c["arrivals"][0][3]["round"] = 1
    c["arrivals"][1][3]["round"] = 2
    c["expect_error"] = "RuntimeError"
    c = add("err_ratio_negative", {"e": (100,)}, torch.float32, 3, [5, -2, 4], 64)
    c["accumulate"] = False
    c["expect_error"] = "AssertionError"
    return cases


def run_reference(case, message, fed):
    """Drive the reference's FedAVGAlgorithm exactly like AggregationServer does."""
    algo = make_hooked_class(fed.FedAVGAlgorithm, case)()
    algo.accumulate = case["accumulate"]
    algo.aggregate_loss = case["aggregate_loss"]
    kinds = case.get("kinds") or ["full"] * len(case["arrivals"])
    for j, ((wid, params, weight, other), kind) in enumerate(zip(case["arrivals"], kinds)):
        if params is None:
            algo.process_worker_data(worker_id=wid, worker_data=None)
            continue
        od = dict(other)
        if kind == "delta":
            # AggregationServer._process_worker_data: data = data.restore(old_parameter)
            dmsg = message.DeltaParameterMessage(delta_parameter={k: v.clone() for k, v in params.items()},
                                                 aggregation_weight=weight, other_data=od)
            msg = dmsg.restore({k: v.clone() for k, v in case["old"].items()})
        else:
            msg = message.ParameterMessage(parameter={k: v.clone() for k, v in params.items()},
                                           aggregation_weight=weight, other_data=od)
            if "old" in case:
                msg.complete(case["old"])
        algo.process_worker_data(worker_id=wid, worker_data=msg)
    return algo.aggregate_worker_data(), getattr(algo, "seen_totals", None)


def _np(t: torch.Tensor) -> np.ndarray:
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def main() -> int:
    if not REF.exists():
        print("reference not present: nothing to generate")
        return 0
    message, _agg, fed = _load_reference()
    arrays: dict[str, np.ndarray] = {}
    manifest = {"generator": "tests/golden/gen_golden.py",
                "reference_files": ["simulation_lib/message.py",
                                    "simulation_lib/algorithm/aggregation_algorithm.py",
                                    "simulation_lib/algorithm/fed_avg_algorithm.py"],
                "cases": []}
    for case in build_cases():
        name = case["name"]
        entry = {
            "name": name,
            "dtype": str(case["dtype"]).replace("torch.", ""),
            "names": list(case["shapes"].keys()),
            "shapes": [list(s) for s in case["shapes"].values()],
            "accumulate": case["accumulate"],
            "aggregate_loss": case["aggregate_loss"],
            "per_tensor_weight": case["per_tensor_weight"],
            "arrivals": [],
            "kinds": case.get("kinds"),
            "weight_mode": case.get("weight_mode"),
            "total_weight_hook": case.get("total_weight_hook"),
        }
        if "old" in case:
            entry["old_keys"] = list(case["old"].keys())
            for k, v in case["old"].items():
                arrays[f"{name}/old/{k}"] = _np(v)
        for j, (wid, params, weight, other) in enumerate(case["arrivals"]):
            a = {"worker_id": wid, "weight": weight, "other_data": other,
                 "keys": None if params is None else list(params.keys())}
            if params is not None:
                for k, v in params.items():
                    arrays[f"{name}/in/{j}/{k}"] = _np(v)
            if case.get("elem_weights") is not None:
                for k, v in case["elem_weights"][j].items():
                    arrays[f"{name}/w/{j}/{k}"] = v.numpy()
            entry["arrivals"].append(a)
        try:
            res, hook_totals = run_reference(case, message, fed)
        except (AssertionError, RuntimeError) as e:
            entry["error"] = type(e).__name__
            if case["expect_error"] is not None:
                assert type(e).__name__ == case["expect_error"], (name, e)
        else:
            assert case["expect_error"] is None, f"{name}: expected {case['expect_error']}"
            entry["error"] = None
            entry["out_keys"] = list(res.parameter.keys())
            entry["out_dtype"] = str(next(iter(res.parameter.values())).dtype).replace("torch.", "")
            for k, v in res.parameter.items():
                arrays[f"{name}/out/{k}"] = v.numpy()
            entry["result_other_data"] = res.other_data
            entry["end_training"] = res.end_training
            entry["in_round"] = res.in_round
            entry["hook_totals"] = hook_totals
        manifest["cases"].append(entry)
        print(f"{name}: {'error ' + entry['error'] if entry['error'] else 'ok'}")
    np.savez_compressed(OUT_DIR / "fedavg_golden.npz", **arrays)
    (OUT_DIR / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=False) + "\n")
    size = (OUT_DIR / "fedavg_golden.npz").stat().st_size
    print(f"wrote {len(manifest['cases'])} cases, {size / 1e6:.2f} MB")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
