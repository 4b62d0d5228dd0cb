"""The caller of the hot path: the server's per-message contract and its poll loop.

Reproduces only what the FedAvg reduce depends on from the reference's
``AggregationServer`` (``simulation_lib/server/aggregation_server.py:111-175``) and
``Server.start`` (``simulation_lib/server/server.py:122-152``):

  * each message is normalised before it reaches the algorithm — a delta is restored
    against the cached global model, a full update is ``complete()``-d with it (:121-129);
  * the algorithm sees ``process_worker_data`` per message and, once every worker has
    reported, ``set_old_parameter`` + ``aggregate_worker_data`` (:130-145);
  * the result is cached as a float64 host copy (``ModelCache``, util/model_cache.py:27-34),
    broadcast, and the algorithm's per-round state is cleared (:147-175).

Model evaluation, early stopping, client selection and session storage are outside the
reduce and not reproduced. Transport is a plain
``multiprocessing`` pipe per worker (the reference uses cyy_naive_lib's pipe topology);
``run_pipe_worker`` is the matching client loop used by the loopback harness (config 1).
"""

from __future__ import annotations

import time
from collections.abc import Callable, Iterable
from multiprocessing.connection import Connection, wait
from typing import Any

import torch

from ..message import (
    Message,
    ParameterMessage,
    is_delta_message,
    is_parameter_message,
    is_parameter_message_base,
    wire_class,
)
from ..quantized import dequantize_parameter, is_quantized


class ModelCache:
    """Last global model as float64 host tensors (util/model_cache.py:10-43)."""

    def __init__(self) -> None:
        self._parameter: dict[str, torch.Tensor] | None = None

    @property
    def has_data(self) -> bool:
        return self._parameter is not None

    @property
    def parameter(self) -> dict[str, torch.Tensor] | None:
        return self._parameter

    def cache_parameter(self, parameter: dict[str, torch.Tensor]) -> None:
        self._parameter = {k: v.detach().to(device="cpu", dtype=torch.float64) for k, v in parameter.items()}

    def get_parameter_diff(self, new_parameter: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
        """new - cached per name (model_cache.py:36-37); a device tensor keeps its device (the
        cached fp64 copy goes to it: the subtraction is one elementwise torch op either way)."""
        assert self._parameter is not None
        return {k: v - self._parameter[k].to(v.device) for k, v in new_parameter.items()}

    def add_parameter_diff(self, parameter_diff: dict[str, torch.Tensor]) -> None:
        """cached += diff per cached name, the diff moved to the host first (model_cache.py:39-43:
        ``v + tensor_to(parameter_diff[k], device="cpu")``; fp64 + the diff's dtype promotes as torch
        does). The reference also re-points its storage file; this cache is in memory only."""
        assert self._parameter is not None
        self._parameter = {k: v + parameter_diff[k].to("cpu") for k, v in self._parameter.items()}


class PipeServerEndpoint:
    """Server end of one duplex pipe per worker."""

    def __init__(self, connections: list[Connection]) -> None:
        self.connections = connections

    @property
    def worker_num(self) -> int:
        return len(self.connections)

    def poll(self, worker_ids: Iterable[int], timeout: float = 1.0) -> dict[int, Any]:
        ids = list(worker_ids)
        ready = wait([self.connections[i] for i in ids], timeout=timeout)
        out: dict[int, Any] = {}
        for i in ids:
            if self.connections[i] in ready:
                out[i] = self.connections[i].recv()
        return out

    def broadcast(self, data: Any, worker_ids: Iterable[int] | None = None) -> None:
        for i in worker_ids if worker_ids is not None else range(self.worker_num):
            self.connections[i].send(data)

    def close(self) -> None:
        for c in self.connections:
            c.close()


class AggregationServer:
    def __init__(
        self,
        algorithm: Any,
        worker_number: int,
        endpoint: PipeServerEndpoint | None = None,
        round_number: int = 1,
        init_parameter: dict[str, torch.Tensor] | None = None,
        config: Any = None,
    ) -> None:
        self.worker_number = worker_number
        self._endpoint = endpoint
        self.round_number = round_number
        self._round_index = 1
        self._stop = False
        self._model_cache = ModelCache()
        self._worker_flag: set[int] = set()
        self.results: list[ParameterMessage] = []
        self.arrivals: list[list[int]] = [[]]  # worker ids in processing order, per result
        self.round_seconds: list[float] = []
        self._round_t0: float | None = None
        algorithm.set_config(config)
        self._algorithm = algorithm
        self._init_parameter = init_parameter

    @property
    def algorithm(self) -> Any:
        return self._algorithm

    @property
    def round_index(self) -> int:
        return self._round_index

    @property
    def current_aggregated_model(self) -> ModelCache:
        return self._model_cache

    def _stopped(self) -> bool:
        return self._round_index > self.round_number or self._stop

    # -- aggregation_server.py:111-141 -------------------------------------------------
    def _process_worker_data(self, worker_id: int, data: Message | None) -> None:
        assert 0 <= worker_id < self.worker_number
        if self._round_t0 is None:
            self._round_t0 = time.perf_counter()
        if data is not None:
            if data.end_training:
                self._stop = True
                if not is_parameter_message_base(data):
                    return
            old_parameter = self._model_cache.parameter
            self._dequantize_if_needed(data)
            if is_delta_message(data):
                assert old_parameter is not None
                if getattr(self._algorithm, "accepts_delta_messages", False):
                    # the algorithm fuses restore() into its fold (fedavg_*_delta)
                    self._algorithm.set_old_parameter(old_parameter)
                else:
                    data = data.restore(old_parameter)
            elif is_parameter_message(data):
                if old_parameter is not None:
                    data.complete(old_parameter)
        self._algorithm.process_worker_data(worker_id=worker_id, worker_data=data)
        self.arrivals[-1].append(worker_id)
        self._worker_flag.add(worker_id)
        if len(self._worker_flag) == self.worker_number:
            result = self._aggregate_worker_data()
            self._send_result(result)
            self._worker_flag.clear()

    def _dequantize_if_needed(self, data: Message) -> None:
        """QuantServerEndpoint.get (topology/quantized_endpoint.py:69-77): quantised payloads
        are dequantised before the algorithm sees them — unless the algorithm folds QSGD
        records itself (FedAVGAlgorithm: dequantisation fused into the kernel). Deltas are
        always dequantised (the delta fold takes dense tensors)."""
        if is_delta_message(data):
            if is_quantized(data.delta_parameter):
                data.delta_parameter = dequantize_parameter(data.delta_parameter)
        elif is_parameter_message(data) and is_quantized(data.parameter):
            if not getattr(self._algorithm, "accepts_quantized_messages", False):
                data.parameter = dequantize_parameter(data.parameter)

    def _aggregate_worker_data(self) -> Message:
        self._algorithm.set_old_parameter(self._model_cache.parameter)
        return self._algorithm.aggregate_worker_data()

    def _send_result(self, result: Message) -> None:
        if is_parameter_message(result):
            self._model_cache.cache_parameter(result.parameter)
            # what crosses the process boundary is the cached host copy
            result = wire_class(result, "ParameterMessage")(
                parameter=self._model_cache.parameter or {},
                end_training=result.end_training,
                in_round=result.in_round,
                other_data=result.other_data,
                is_initial=result.is_initial,
            )
            self.results.append(result)
            self.arrivals.append([])
        if self._round_t0 is not None:
            self.round_seconds.append(time.perf_counter() - self._round_t0)
            self._round_t0 = None
        if self._endpoint is not None:
            self._endpoint.broadcast(result)
        if not result.in_round:
            self._round_index += 1
        self._algorithm.clear_worker_data()

    # -- server.py:122-152 (poll loop) -------------------------------------------------
    def start(self) -> None:
        assert self._endpoint is not None
        if self._init_parameter is not None:
            self._send_result(ParameterMessage(parameter=self._init_parameter, in_round=True, is_initial=True))
        pending: set[int] = set()
        while not self._stopped():
            if not pending:
                pending = set(range(self._endpoint.worker_num))
            for worker_id, data in self._endpoint.poll(pending).items():
                self._process_worker_data(worker_id=worker_id, data=data)
                pending.discard(worker_id)
        self._algorithm.exit()


def run_pipe_worker(
    conn: Connection,
    make_update: Callable[[int], ParameterMessage],
    round_number: int,
    receive_initial: bool = False,
) -> None:
    """Client loop: send one update per round, wait for the aggregated model."""
    if receive_initial:
        conn.recv()
    for r in range(round_number):
        conn.send(make_update(r))
        conn.recv()
    conn.close()
