"""Where a bench step's time goes: host call, kernel, NaN-flag readback (GPU box)."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, OutputTable  # noqa: E402

dev = torch.device("cuda", 0)
layout = resnet18_layout()
K = 64
buckets, views = make_clients(layout, 0, K, dev, torch.float32)
w = dataset_size_weights(K)
table = ClientTable(layout.num_segments)
for row, wk in zip(views, w):
    table.add_client(row, [wk] * layout.num_segments)
offs, padded = layout.padded_offsets(4)
flat = torch.empty(padded, dtype=torch.float32, device=dev)
outs = OutputTable([flat[o:o + m] for o, m in zip(offs, layout.numels)], layout, dev, torch.float32)
ctx = FedAvgContext(layout, dev)
for _ in range(5):
    ctx.aggregate(table, torch.float32, outs, torch.float32)
    ctx.raise_on_nan()
torch.cuda.synchronize()
n = 50
t_call = t_check = 0.0
ctx.prof_enable(True)
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    ctx.aggregate(table, torch.float32, outs, torch.float32)
    b = time.perf_counter()
    ctx.raise_on_nan()
    c = time.perf_counter()
    t_call += b - a
    t_check += c - b
total = time.perf_counter() - t0
ms, launches = ctx.prof_collect()
print(f"step {total / n * 1e3:.4f} ms | host call {t_call / n * 1e3:.4f} ms | check (incl. wait) {t_check / n * 1e3:.4f} ms | kernel {ms / launches:.4f} ms")
# pure launch loop without per-step check (throughput ceiling of back-to-back rounds)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    ctx.aggregate(table, torch.float32, outs, torch.float32)
torch.cuda.synchronize()
print(f"back-to-back aggregate without per-step check: {(time.perf_counter() - t0) / n * 1e3:.4f} ms/step")
