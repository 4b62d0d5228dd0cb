"""Where do the ~19 us between two headline rounds go? (GPU box, 1 GPU)

One round = plan.run() (one launch) + ctx.raise_on_nan() (stream sync + flag read). Modes,
interleaved: the default HIP wait, a Python busy-poll on hipStreamQuery before the check, and
the same after hipSetDeviceFlags(hipDeviceScheduleSpin). Prints median step and kernel ms.
"""
import ctypes
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, OutputTable  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    layout = resnet18_layout()
    K = 64
    _, views = make_clients(layout, 0, K, dev, torch.float32)
    table = ClientTable(layout.num_segments)
    for row, w in zip(views, dataset_size_weights(K)):
        table.add_client(row, [w] * layout.num_segments)
    offs, padded = layout.padded_offsets(4)
    flat = torch.empty(padded, dtype=torch.float32, device=dev)
    outs = OutputTable([flat[o:o + m] for o, m in zip(offs, layout.numels)], layout, dev, torch.float32)
    ctx = FedAvgContext(layout, dev)
    plan = ctx.plan(table, torch.float32, outs, torch.float32)
    hip = ctypes.CDLL("libamdhip64.so")
    stream = ctx.stream

    def step_default():
        plan.run()
        ctx.raise_on_nan()

    def step_poll():
        plan.run()
        while hip.hipStreamQuery(stream) != 0:
            pass
        ctx.raise_on_nan()

    modes = {"default": step_default, "poll": step_poll}
    res = {m: [] for m in modes}
    for _ in range(20):
        step_default()
    for rep in range(7):
        for m, fn in modes.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                fn()
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) / 50 * 1e3)
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    res["spin_flag"] = []
    for rep in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            step_default()
        torch.cuda.synchronize()
        res["spin_flag"].append((time.perf_counter() - t0) / 50 * 1e3)
    ctx.prof_enable(True)
    for _ in range(50):
        step_default()
    ctx.prof_enable(False)
    kms, n = ctx.prof_collect()
    print(f"hipSetDeviceFlags(spin) rc={rc}")
    for m, v in res.items():
        print(f"{m:10s} step median {statistics.median(v):.4f} ms  min {min(v):.4f}")
    print(f"kernel mean {kms / max(n, 1):.4f} ms over {n} launches")


if __name__ == "__main__":
    main()
