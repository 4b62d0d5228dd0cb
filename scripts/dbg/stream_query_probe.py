"""Debug probe: is the caller's stream idle (hipStreamQuery) after a dynamic wave's close + sync?"""
import ctypes
import os

os.environ.setdefault("FEDAVG_DYN_IDLE_US", "1000000")
import torch

from distributed_learning_simulation_lib_amd._staging import NativeClientTable
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext, ModelLayout, OutputTable

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
layout = ModelLayout.flat(100_000)
xs = [torch.randn(100_000, device=dev) for _ in range(7)]
table = NativeClientTable(1, 0)
for k, x in enumerate(xs):
    table.add_client([x], [float(3 + k)])
out = torch.empty(100_000, dtype=torch.float64, device=dev)
ctx = FedAvgContext(layout, dev)
outs = OutputTable([out], layout, dev, torch.float64)
s = ctx.stream
print("stream handle", ctx.stream, torch.cuda.current_stream().cuda_stream)
for rnd in range(3):
    ctx.dyn_open(torch.float32, 16)
    ctx.dyn_publish(table)
    print("close", ctx.dyn_close(outs, torch.float64))
    print(" query right after close", hip.hipStreamQuery(s))
    hip.hipStreamSynchronize(s)
    print(" query after sync", hip.hipStreamQuery(s), hip.hipStreamQuery(s))
    ctx.raise_on_nan()
    print(" query after raise_on_nan", hip.hipStreamQuery(s))
    ctx.reset()
    print(" query after reset", hip.hipStreamQuery(s))
ctx.aggregate(table, torch.float32, outs, torch.float64)
ctx.raise_on_nan()
print("static round: query after raise_on_nan", hip.hipStreamQuery(s))
ctx.close()
