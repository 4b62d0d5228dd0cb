from .aggregation_algorithm import AggregationAlgorithm
from .fed_avg_algorithm import FedAVGAlgorithm

__all__ = ["AggregationAlgorithm", "FedAVGAlgorithm"]
