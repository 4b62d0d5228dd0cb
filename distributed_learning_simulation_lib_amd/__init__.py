"""MI355X-native server-side FedAvg aggregation for distributed_learning_simulation_lib.

The hot path — the weighted reduction of N clients' parameter tensors into one global model
(reference ``simulation_lib/algorithm/fed_avg_algorithm.py``) — runs in hand-written gfx950
HIP kernels behind the C ABI of ``include/fedavg_hip.h``; this package is the host side that
keeps the reference's plugin surface.
"""

from .algorithm import AggregationAlgorithm, FedAVGAlgorithm, PersonalizedFedAVGAlgorithm
from .algorithm_repository import AlgorithmRepository
from .fedavg import ClientTable, FedAvgContext, ModelLayout, NaNAggregationError
from .message import (
    DeltaParameterMessage,
    FeatureMessage,
    Message,
    ModelParameter,
    MultipleWorkerMessage,
    ParameterMessage,
    ParameterMessageBase,
    get_message_size,
)

__all__ = [
    "AggregationAlgorithm",
    "AlgorithmRepository",
    "ClientTable",
    "DeltaParameterMessage",
    "FeatureMessage",
    "FedAVGAlgorithm",
    "FedAvgContext",
    "Message",
    "ModelLayout",
    "ModelParameter",
    "MultipleWorkerMessage",
    "NaNAggregationError",
    "ParameterMessage",
    "ParameterMessageBase",
    "PersonalizedFedAVGAlgorithm",
    "get_message_size",
]


def _register_builtin() -> None:
    """The reference registers "fed_avg" at import (common_method/__init__.py:6-11). The
    client class is the simulator's worker, outside this package: it is left as None."""
    if not AlgorithmRepository.has_algorithm("fed_avg"):
        from .server import AggregationServer

        AlgorithmRepository.register_algorithm(
            algorithm_name="fed_avg",
            client_cls=None,  # type: ignore[arg-type]
            server_cls=AggregationServer,
            algorithm_cls=FedAVGAlgorithm,
        )


_register_builtin()
