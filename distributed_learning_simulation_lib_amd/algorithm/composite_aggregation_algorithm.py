"""A chain of aggregation algorithms behind one plugin object.

Same surface and semantics as the reference's ``CompositeAggregationAlgorithm``
(``simulation_lib/algorithm/composite_aggregation_algorithm.py:10-69``): configuration and the
old global model are forwarded to every member; the first member whose
``process_worker_data`` accepts an arrival handles the rest of the round; ``aggregate_worker_data``
asks that member and releases it; an arrival nobody accepts raises ``NotImplementedError``.
Pure host logic: the members (e.g. the HIP ``FedAVGAlgorithm``) do the reduce.
"""

from __future__ import annotations

from typing import Any

from ..message import Message, ModelParameter
from .aggregation_algorithm import AggregationAlgorithm


class CompositeAggregationAlgorithm(AggregationAlgorithm):
    def __init__(self) -> None:
        super().__init__()
        self.__algorithms: list[AggregationAlgorithm] = []
        self.__used_algorithm: AggregationAlgorithm | None = None

    def prepend_algorithm(self, algorithm: AggregationAlgorithm) -> None:
        self.__algorithms.insert(0, algorithm)

    def append_algorithm(self, algorithm: AggregationAlgorithm) -> None:
        self.__algorithms.append(algorithm)

    # :22-30
    def set_old_parameter(self, old_parameter: ModelParameter) -> None:
        for algorithm in self.__algorithms:
            algorithm.set_old_parameter(old_parameter=old_parameter)

    def set_config(self, config: Any) -> None:
        for algorithm in self.__algorithms:
            algorithm.set_config(config=config)

    # :32-52
    def process_worker_data(self, worker_id: int, worker_data: Message | None) -> bool:
        if self.__used_algorithm is not None:
            res = self.__used_algorithm.process_worker_data(worker_id=worker_id, worker_data=worker_data)
            assert res
            return True
        for algorithm in self.__algorithms:
            if algorithm.process_worker_data(worker_id=worker_id, worker_data=worker_data):
                self.__used_algorithm = algorithm
                return True
        raise NotImplementedError("Failed to process_worker_data")

    # :54-59
    def aggregate_worker_data(self) -> Any:
        assert self.__used_algorithm is not None
        res = self.__used_algorithm.aggregate_worker_data()
        self.__used_algorithm = None
        return res

    # :61-69
    def clear_worker_data(self) -> None:
        for algorithm in self.__algorithms:
            algorithm.clear_worker_data()

    def exit(self) -> None:
        for algorithm in self.__algorithms:
            algorithm.exit()
