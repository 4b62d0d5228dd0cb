from .aggregation_algorithm import AggregationAlgorithm
from .fed_avg_algorithm import FedAVGAlgorithm
from .personalized_aggregation_algorithm import PersonalizedFedAVGAlgorithm

__all__ = ["AggregationAlgorithm", "FedAVGAlgorithm", "PersonalizedFedAVGAlgorithm"]
