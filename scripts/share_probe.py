"""What the plugin round's dynamic wave costs a GPU shared with another process's kernels (GPU box).

A child process keeps the GPU busy with bf16 GEMMs (the stand-in for workers training on the same
GPU, as in the reference's simulator: workers and server share the node's GPUs) and reports its
GEMM rate over fixed windows; the parent runs 64 x ResNet-18 fp32 plugin rounds
(FedAVGAlgorithm.process_worker_data x 64 + aggregate_worker_data, device-resident updates) in the
same windows, with the dynamic wave on and off, and alone. One JSON line:

    python scripts/share_probe.py [seconds per window]
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def gemm_child(conn, n: int) -> None:
    import torch

    dev = torch.device("cuda", 0)
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    conn.send("ready")
    while True:
        cmd = conn.recv()
        if cmd == "stop":
            break
        seconds = float(cmd)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < seconds:
            for _ in range(4):
                torch.matmul(a, b, out=c)
            torch.cuda.synchronize()
            k += 4
        el = time.perf_counter() - t0
        conn.send({"gemms": k, "seconds": el, "tflops": 2.0 * n**3 * k / el / 1e12})


def main() -> None:
    import torch

    from bench import dataset_size_weights, make_clients, resnet18_layout
    from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage

    window = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    dev = torch.device("cuda", 0)
    layout = resnet18_layout()
    N = 64
    _, views = make_clients(layout, 0, N, dev, torch.float32)
    params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
    weights = dataset_size_weights(N)

    def rounds(algo, seconds: float) -> dict:
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < seconds:
            for wid, (p, w) in enumerate(zip(params, weights)):
                algo.process_worker_data(wid, ParameterMessage(parameter=dict(p), aggregation_weight=w))
            algo.aggregate_worker_data()
            algo.clear_worker_data()
            k += 1
        el = time.perf_counter() - t0
        return {"rounds": k, "ms_per_round": round(el / k * 1e3, 4)}

    algos = {"dyn": FedAVGAlgorithm(device=dev, dynamic_wave=True),
             "static": FedAVGAlgorithm(device=dev, dynamic_wave=False)}
    for a in algos.values():  # warm
        rounds(a, 0.3)
    out: dict = {"window_s": window}
    for name, a in algos.items():
        out[f"plugin_alone_{name}"] = rounds(a, window)
    ctx = mp.get_context("spawn")
    parent, child = ctx.Pipe()
    p = ctx.Process(target=gemm_child, args=(child, 8192))
    p.start()
    assert parent.recv() == "ready"
    parent.send(str(window))
    out["gemm_alone"] = parent.recv()
    for name, a in algos.items():
        parent.send(str(window))
        out[f"plugin_shared_{name}"] = rounds(a, window)
        out[f"gemm_shared_{name}"] = parent.recv()
    parent.send("stop")
    p.join(timeout=60)
    for a in algos.values():
        out.setdefault("dyn_stats", {})
        a.exit()
    out["dyn_stats"] = algos["dyn"].dyn_stats
    g0 = out["gemm_alone"]["tflops"]
    out["summary"] = {
        "gemm_rate_with_plugin_dyn": round(out["gemm_shared_dyn"]["tflops"] / g0, 3),
        "gemm_rate_with_plugin_static": round(out["gemm_shared_static"]["tflops"] / g0, 3),
        "plugin_round_shared_dyn_ms": out["plugin_shared_dyn"]["ms_per_round"],
        "plugin_round_shared_static_ms": out["plugin_shared_static"]["ms_per_round"],
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    main()
