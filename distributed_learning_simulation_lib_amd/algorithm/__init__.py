from .aggregation_algorithm import AggregationAlgorithm
from .composite_aggregation_algorithm import CompositeAggregationAlgorithm
from .fed_avg_algorithm import FedAVGAlgorithm
from .personalized_aggregation_algorithm import PersonalizedFedAVGAlgorithm

__all__ = ["AggregationAlgorithm", "CompositeAggregationAlgorithm", "FedAVGAlgorithm", "PersonalizedFedAVGAlgorithm"]
