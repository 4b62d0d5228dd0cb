"""ORACLE — test infrastructure only: the reference's CPU op sequence, for the CPU baseline.

``bench.py``'s ``cpu_baseline`` leg times this. It issues exactly the torch CPU operations the
reference's streaming FedAvg issues per client tensor
(simulation_lib/algorithm/fed_avg_algorithm.py:34-62 and :92-97):

    assert not x.isnan().any()          # :35
    tmp = x.to(float64) * w             # :54
    acc = tmp / acc += tmp              # :55-58
    ...
    assert not acc.isnan().any(); out = acc / W; assert not out.isnan().any()   # :93-97

so its timing is the reference's CPU path on the same host (kind "port" in bench.py), with
message plumbing excluded. Parity with the reference is pinned through
``oracle/fedavg_oracle.py`` in ``tests/test_oracle_golden.py``.
"""

from __future__ import annotations

import torch


class RefOpsFedAvg:
    def __init__(self) -> None:
        self.acc: dict[str, torch.Tensor] = {}
        self.totals: dict[str, float] = {}

    def add(self, parameter: dict[str, torch.Tensor], weight: float) -> None:
        for name, x in parameter.items():
            assert not x.isnan().any().cpu()
            tmp = x.to(dtype=torch.float64) * weight
            if name not in self.acc:
                self.acc[name] = tmp
            else:
                self.acc[name] += tmp
            self.totals[name] = self.totals.get(name, 0) + weight

    def finish(self) -> dict[str, torch.Tensor]:
        out = {}
        for k, v in self.acc.items():
            assert not v.isnan().any().cpu()
            out[k] = v / self.totals[k]
            assert not out[k].isnan().any().cpu()
        self.acc, self.totals = {}, {}
        return out


class RefFedAvgAlgorithm:
    """The reference's FedAVGAlgorithm call sequence (fed_avg_algorithm.py:20-113) over message
    objects, in the reference's torch CPU ops: ``process_worker_data`` per arrival (NaN assert,
    weighted fp64 fold, payload released, :20-64), ``aggregate_worker_data`` at the end (NaN
    asserts, divide, other_data check, first-arrival flags, :76-113). bench.py's cpu_baseline
    times process_worker_data x N + aggregate_worker_data on pre-built messages."""

    def __init__(self) -> None:
        self.ops = RefOpsFedAvg()
        self.all_worker_data: dict = {}

    def process_worker_data(self, worker_id: int, worker_data) -> bool:
        self.all_worker_data[worker_id] = worker_data
        if worker_data is None:
            return True
        self.ops.add(worker_data.parameter, worker_data.aggregation_weight)
        worker_data.parameter = {}  # :63-64
        return True

    def aggregate_worker_data(self) -> dict:
        parameter = self.ops.finish()
        other: dict = {}
        for msg in self.all_worker_data.values():
            for k, v in msg.other_data.items():
                if k in other and other[k] != v:
                    raise RuntimeError(f"different values on key {k}")
                other.setdefault(k, v)
        first = next(iter(self.all_worker_data.values()))
        return {"parameter": parameter, "other_data": other, "in_round": first.in_round,
                "end_training": first.end_training}


class RefOpsPersonalized:
    """The reference's PersonalizedFedAVG op sequence (personalized_aggregation_algorithm.py:23-57)
    in torch CPU ops, for bench.py's personalized cpu_baseline: every arrival is deep-copied into
    each other receiver's FedAvg (copy.deepcopy, :38-40) and folded there (RefOpsFedAvg above);
    the centralized model is the equal-weight weighted_avg of the receivers' results (:51-53,
    aggregation_algorithm.py:63-74)."""

    def __init__(self, worker_weights: dict[int, dict[int, float]]) -> None:
        self.worker_weights = worker_weights
        self.algos = {j: RefOpsFedAvg() for j in worker_weights}

    def add(self, worker_id: int, parameter: dict[str, torch.Tensor]) -> None:
        for j, algo in self.algos.items():
            if j == worker_id:
                continue
            copy = {k: v.clone() for k, v in parameter.items()}  # copy.deepcopy of the message
            algo.add(copy, self.worker_weights[j].get(worker_id, 0))

    def finish(self) -> tuple[dict[int, dict[str, torch.Tensor]], dict[str, torch.Tensor]]:
        results = {j: a.finish() for j, a in self.algos.items()}
        c = 1 / len(results)
        central: dict[str, torch.Tensor] = {}
        for r in results.values():
            d = {k: v.to(dtype=torch.float64) * c for k, v in r.items()}
            if not central:
                central = d
            else:
                for k in central:
                    central[k] += d[k]
        for v in central.values():
            assert not v.isnan().any().cpu()
        return results, central
