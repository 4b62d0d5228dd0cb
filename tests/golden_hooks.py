"""The overridden FedAVGAlgorithm hooks of the golden cases (test-only).

One definition, used both by ``tests/golden/gen_golden.py`` (subclassing the reference's own
FedAVGAlgorithm to produce the expected outputs) and by the GPU tests (subclassing the HIP
FedAVGAlgorithm), so both run the very same hook code:

  * per_tensor_weight: ``_get_weight`` returns a number per (client, tensor);
  * weight_mode "scalar_tensor_float32/64": a fresh 0-dim tensor of that dtype;
  * weight_mode "elementwise_float32/64": a tensor of the parameter's shape
    (``elem_weights[arrival][name]``, the arrival being ``aggregation_weight``);
  * total_weight_hook "scaled": ``_apply_total_weight`` = (x * 3) / (total + 1), recording the
    totals it is handed in ``seen_totals``.
"""

from __future__ import annotations

import torch


def make_hooked_class(base, case):
    """The case's subclass of a FedAVGAlgorithm (the reference's, or the HIP one in the GPU tests):
    the overridden _get_weight / _apply_total_weight hooks the case names. Shared by the
    generator and tests/test_gpu_hooks.py so both run the very same hook code."""
    ptw = case.get("per_tensor_weight")
    mode = case.get("weight_mode")
    hook = case.get("total_weight_hook")
    elem = case.get("elem_weights")
    if ptw is None and mode is None and hook is None:
        return base

    def _get_weight(self, worker_data, name, parameter):
        if ptw is not None:
            return ptw[name][int(worker_data.aggregation_weight)]
        if mode == "scalar_tensor_float32":
            return torch.tensor(worker_data.aggregation_weight, dtype=torch.float32)
        if mode == "scalar_tensor_float64":
            return torch.tensor(worker_data.aggregation_weight, dtype=torch.float64)
        if mode is not None and mode.startswith("elementwise"):
            # a fresh copy: the reference adds the later weights into the first one in place
            return elem[int(worker_data.aggregation_weight)][name].clone()
        return base._get_weight(self, worker_data=worker_data, name=name, parameter=parameter)

    def _apply_total_weight(self, name, parameter, total_weight):
        if not hasattr(self, "seen_totals"):
            self.seen_totals = {}
        self.seen_totals[name] = float(total_weight) if not isinstance(total_weight, torch.Tensor) \
            or total_weight.numel() == 1 else total_weight.double().sum().item()
        return (parameter * 3.0) / (total_weight + 1)

    members = {}
    if ptw is not None or mode is not None:
        members["_get_weight"] = _get_weight
    if hook is not None:
        members["_apply_total_weight"] = _apply_total_weight
    return type("Hooked", (base,), members)
