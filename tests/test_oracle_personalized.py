"""The PersonalizedFedAVG oracle against the reference's own outputs (parity pin, CPU-only)."""

import pytest

from oracle.fedavg_oracle import OracleMessage
from oracle.personalized_oracle import OraclePersonalizedFedAvg
from tests.golden_io import bits_equal, load_personalized

CASES = load_personalized()


def run_oracle(case):
    algo = OraclePersonalizedFedAvg()
    algo.set_worker_weights({j: dict(v) for j, v in case.worker_weights.items()})
    for a in case.arrivals:
        msg = None
        if a.arrays is not None:
            msg = OracleMessage(parameter=dict(a.arrays), other_data=dict(a.other_data), dtype=case.dtype)
        algo.process_worker_data(a.worker_id, msg)
    return algo.aggregate_worker_data()


@pytest.mark.parametrize("name", sorted(CASES))
def test_personalized_oracle_matches_reference(name):
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_oracle(case)
        return
    res = run_oracle(case)
    assert list(res.worker_data) == [r["worker_id"] for r in case.meta["receivers"]]
    for r in case.meta["receivers"]:
        got = res.worker_data[r["worker_id"]]
        assert list(got.parameter) == r["keys"]
        for k, want in case.expected[r["worker_id"]].items():
            assert bits_equal(got.parameter[k], want), f"{name}/{r['worker_id']}/{k}"
        assert got.other_data == r["other_data"]
        assert (got.in_round, got.end_training) == (r["in_round"], r["end_training"])
    assert list(res.centralized_parameter) == case.meta["central_keys"]
    for k, want in case.central.items():
        assert bits_equal(res.centralized_parameter[k], want), f"{name}/central/{k}"


def test_personalized_golden_covers_the_edge_cases():
    for required in ("p_order", "p_subset", "p_skipped", "p_signed_zero", "p_n64", "p_n80",
                     "p_n3_f16", "p_n3_bf16", "p_n3_f64", "p_err_nan_input", "p_err_zero_total",
                     "p_err_no_data", "p_err_other_data", "p_err_inf_zero_weight"):
        assert required in CASES
