"""Test-only adapters: the oracle behind the server's algorithm interface, worker payloads."""

from __future__ import annotations

import tempfile

import numpy as np
import torch

from distributed_learning_simulation_lib_amd.message import ParameterMessage
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage


class OracleAlgorithm:
    """The CPU oracle wearing the AggregationAlgorithm protocol (checker for server tests)."""

    def __init__(self) -> None:
        self.o = OracleFedAvg()
        self.old = None
        self.config = None

    def set_config(self, config) -> None:
        self.config = config

    def set_old_parameter(self, old_parameter) -> None:
        self.old = old_parameter

    def process_worker_data(self, worker_id, worker_data) -> bool:
        if worker_data is None:
            return self.o.process_worker_data(worker_id, None)
        msg = OracleMessage(
            parameter={k: v.numpy() for k, v in worker_data.parameter.items()},
            aggregation_weight=worker_data.aggregation_weight,
            other_data=dict(worker_data.other_data),
            in_round=worker_data.in_round,
            end_training=worker_data.end_training,
        )
        return self.o.process_worker_data(worker_id, msg)

    def aggregate_worker_data(self):
        r = self.o.aggregate_worker_data()
        return ParameterMessage(
            parameter={k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in r.parameter.items()},
            in_round=r.in_round,
            end_training=r.end_training,
            other_data=r.other_data,
        )

    def clear_worker_data(self) -> None:
        self.o = OracleFedAvg()

    def exit(self) -> None:
        pass


def config1_update(worker: int, round_idx: int, numel: int = 1_000_000) -> ParameterMessage:
    """BASELINE config 1 payload: x ~ N(0,1) seeded 1234+worker (+round), fp32, dataset-size weight."""
    g = torch.Generator().manual_seed(1234 + worker + 1000 * round_idx)
    weight = int(np.random.default_rng(99).integers(100, 5001, size=16)[worker])
    return ParameterMessage(parameter={"model": torch.randn(numel, generator=g)}, aggregation_weight=weight)


def rendezvous_url() -> str:
    """A fresh file:// rendezvous for a multi-process test group (no TCP port to race for)."""
    return "file://" + tempfile.mkdtemp(prefix="fedavg_rdzv_") + "/store"
