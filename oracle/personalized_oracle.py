"""ORACLE — test infrastructure only, never product code.

numpy float64 restatement of the reference's ``PersonalizedFedAVGAlgorithm``
(simulation_lib/algorithm/personalized_aggregation_algorithm.py:9-57): one FedAvg per
receiver j, fed every other worker's update with the weight ``worker_weights[j].get(i, 0)``
(:29-43), then the centralized model = the equal-weight ``weighted_avg`` of the receivers'
results in receiver key order (:45-57, aggregation_algorithm.py:51-76).

Each receiver's FedAvg is ``OracleFedAvg`` (oracle/fedavg_oracle.py, pinned against the
reference). This module is pinned by ``tests/test_oracle_golden.py`` against
``tests/golden/personalized_golden.npz`` (generated from the reference's own code by
``tests/golden/gen_personalized.py``).
"""

from __future__ import annotations

import copy
from dataclasses import dataclass
from typing import Any

import numpy as np

from .fedavg_oracle import OracleFedAvg, OracleMessage, OracleResult, weighted_avg


@dataclass
class OraclePersonalizedResult:
    """MultipleWorkerMessage(worker_data=..., other_data={"centralized_parameter": ...}) (:54-57)."""

    worker_data: dict[int, OracleResult]
    centralized_parameter: dict[str, np.ndarray]


class OraclePersonalizedFedAvg:
    def __init__(self) -> None:
        self.worker_weights: dict[int, dict[int, Any]] = {}
        self.algorithms: dict[int, OracleFedAvg] = {}

    # :15-21
    def set_worker_weights(self, worker_weights: dict[int, dict[int, Any]]) -> None:
        assert not self.worker_weights and not self.algorithms
        self.worker_weights = worker_weights
        self.algorithms = {j: OracleFedAvg() for j in worker_weights}

    # :23-43
    def process_worker_data(self, worker_id: int, msg: OracleMessage | None) -> bool:
        assert self.worker_weights and self.algorithms
        for j in self.worker_weights:
            if j == worker_id:
                continue
            w = self.worker_weights[j].get(worker_id, 0)
            m = None
            if msg is not None:
                m = copy.deepcopy(msg)
                m.aggregation_weight = w
            self.algorithms[j].process_worker_data(worker_id, m)
        return True

    # :45-57
    def aggregate_worker_data(self) -> OraclePersonalizedResult:
        results = {j: a.aggregate_worker_data() for j, a in self.algorithms.items()}
        as_msgs = {j: OracleMessage(parameter=r.parameter) for j, r in results.items()}
        central = weighted_avg(as_msgs, 1 / len(as_msgs))
        return OraclePersonalizedResult(results, central)
