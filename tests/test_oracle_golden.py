"""The CPU oracle restatement against the reference's own outputs (parity pin, CPU-only)."""

import pytest

from oracle.fedavg_oracle import OracleFedAvg, OracleMessage, complete, restore
from tests.golden_io import bits_equal, load_golden

CASES = load_golden()


def run_oracle(case):
    ptw = case.per_tensor_weight
    get_weight = None
    if ptw is not None:
        def get_weight(m, name):
            return ptw[name][int(m.aggregation_weight)]
    algo = OracleFedAvg(accumulate=case.accumulate, aggregate_loss=case.aggregate_loss, get_weight=get_weight)
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


def test_golden_covers_the_edge_cases():
    names = set(CASES)
    for required in ("skipped", "order_rev", "ratio_path", "signed_zero", "negative_weight",
                     "per_tensor_weight", "missing_key", "n8_f16", "n8_bf16", "n8_f64",
                     "err_nan_input", "err_inf_minus_inf", "err_zero_total_weight",
                     "err_other_data_mismatch", "err_ratio_negative"):
        assert required in names
