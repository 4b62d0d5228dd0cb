"""Workgroup-tail probe: the fused fp32 kernel's per-byte rate vs the number of 8192-element tiles
(one workgroup each, one resident workgroup per CU): flat layouts of k * 256 tiles and in between.

Usage (GPU box): python scripts/tail_probe.py [clients]
"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from bench import dataset_size_weights, make_clients  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
w = dataset_size_weights(K)
for tiles in (1024, 1152, 1280, 1300, 1408, 1427, 1536, 1664):
    layout = ModelLayout.flat(tiles * 8192)
    buckets, views = make_clients(layout, 0, K, dev, torch.float32)
    table = ClientTable(1)
    for row, wk in zip(views, w):
        table.add_client(row, [wk])
    out = [torch.empty(layout.total_numel, dtype=torch.float32, device=dev)]
    ctx = FedAvgContext(layout, dev)
    plan = ctx.plan(table, torch.float32, out, torch.float32)
    for _ in range(3):
        plan.run()
    ctx.prof_collect()
    times = []
    for _ in range(5):
        ctx.prof_enable(True)
        for _ in range(10):
            plan.run()
        ctx.prof_enable(False)
        ms, n = ctx.prof_collect()
        times.append(ms / n)
    ms = float(np.median(times))
    nbytes = (K + 1) * layout.total_numel * 4
    print(f"tiles {tiles:5d} ({tiles / 256:.2f} per CU): {ms:.4f} ms  {nbytes / ms / 1e9:.1f} GB/s", flush=True)
    del buckets, views, table, out, plan, ctx
    torch.cuda.empty_cache()
