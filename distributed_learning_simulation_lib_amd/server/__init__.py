from .aggregation_server import AggregationServer, ModelCache, PipeServerEndpoint, run_pipe_worker

__all__ = ["AggregationServer", "ModelCache", "PipeServerEndpoint", "run_pipe_worker"]
