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
