"""The CPU oracle restatement against the reference's own outputs (parity pin, CPU-only)."""

import numpy as np
import pytest

from oracle.fedavg_oracle import OracleFedAvg, OracleMessage, complete, restore
from tests.golden_io import bits_equal, load_golden

CASES = load_golden()


def oracle_hooks(case):
    """The golden case's overridden hooks (tests/golden/gen_golden.py make_hooked_class) in numpy."""
    ptw, mode = case.per_tensor_weight, case.weight_mode
    get_weight = apply_total = None
    if ptw is not None:
        def get_weight(m, name):
            return ptw[name][int(m.aggregation_weight)]
    elif mode in ("scalar_tensor_float32", "scalar_tensor_float64"):
        dt = np.float32 if mode.endswith("32") else np.float64

        def get_weight(m, name):
            return dt(m.aggregation_weight)
    elif mode is not None and mode.startswith("elementwise"):
        rows = {a.weight: a.elem_weights for a in case.arrivals if a.elem_weights is not None}

        def get_weight(m, name):
            return np.array(rows[m.aggregation_weight][name], copy=True)
    if case.total_weight_hook == "scaled":
        seen = {}

        def apply_total(name, v, total):
            seen[name] = float(total)
            return (v * 3.0) / (total + 1)
        apply_total.seen = seen
    return get_weight, apply_total


def run_oracle(case):
    get_weight, apply_total = oracle_hooks(case)
    algo = OracleFedAvg(accumulate=case.accumulate, aggregate_loss=case.aggregate_loss, get_weight=get_weight,
                        apply_total_weight=apply_total)
    kinds = case.kinds or ["full"] * len(case.arrivals)
    for a, kind in zip(case.arrivals, kinds):
        if a.arrays is None:
            algo.process_worker_data(a.worker_id, None)
            continue
        params = dict(a.arrays)
        if kind == "delta":
            params = restore(params, case.old)
        elif case.old is not None:
            complete(params, case.old)
        msg = OracleMessage(parameter=params, aggregation_weight=a.weight,
                            other_data=dict(a.other_data), dtype=case.dtype)
        algo.process_worker_data(a.worker_id, msg)
    return algo.aggregate_worker_data()


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference(name):
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_oracle(case)
        return
    res = run_oracle(case)
    assert list(res.parameter.keys()) == case.meta["out_keys"]
    for k, want in case.expected.items():
        assert bits_equal(res.parameter[k], want), f"{name}/{k}"
    assert res.other_data == case.meta["result_other_data"]
    assert res.in_round == case.meta["in_round"] and res.end_training == case.meta["end_training"]


def test_total_weight_hook_sees_the_reference_totals():
    case = CASES["total_weight_hook"]
    _, apply_total = oracle_hooks(case)
    get_weight, _ = oracle_hooks(case)
    algo = OracleFedAvg(get_weight=get_weight, apply_total_weight=apply_total)
    for a in case.arrivals:
        algo.process_worker_data(a.worker_id, OracleMessage(parameter=dict(a.arrays), aggregation_weight=a.weight))
    algo.aggregate_worker_data()
    assert apply_total.seen == case.meta["hook_totals"]


def test_golden_covers_the_edge_cases():
    names = set(CASES)
    for required in ("skipped", "order_rev", "ratio_path", "signed_zero", "negative_weight",
                     "per_tensor_weight", "missing_key", "n8_f16", "n8_bf16", "n8_f64",
                     "err_nan_input", "err_inf_minus_inf", "err_zero_total_weight",
                     "err_other_data_mismatch", "err_ratio_negative"):
        assert required in names
