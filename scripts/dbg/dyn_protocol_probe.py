"""Debug probe: the dynamic wave's C-ABI protocol in variants, printing (folded, finalized)."""
import os
import time

os.environ.setdefault("FEDAVG_DYN_IDLE_US", "1000000")
import torch

from distributed_learning_simulation_lib_amd import _native
from distributed_learning_simulation_lib_amd._staging import NativeClientTable
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext, ModelLayout, OutputTable

dev = torch.device("cuda", 0)
for numel in (10_000, 100_000):
    layout = ModelLayout.flat(numel)
    xs = [torch.randn(numel, device=dev) for _ in range(7)]
    table = NativeClientTable(1, 0)
    for k, x in enumerate(xs):
        table.add_client([x], [float(3 + k)])
    out = torch.empty(numel, dtype=torch.float64, device=dev)
    for variant in ("plain", "failed_launch", "nosync", "acc"):
        ctx = FedAvgContext(layout, dev)
        outs = OutputTable([out], layout, dev, torch.float64)
        t0 = time.perf_counter()
        ctx.dyn_open(torch.float32, 16)
        if variant == "failed_launch":
            try:
                ctx.accumulate(table, torch.float32)
            except _native.NativeError as e:
                print("  refused:", e)
        if variant != "nosync":
            torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        pub = ctx.dyn_publish(table)
        t2 = time.perf_counter()
        time.sleep(0.01)
        res = ctx.dyn_close(None if variant == "acc" else outs, torch.float64)
        t3 = time.perf_counter()
        print(f"numel={numel} {variant}: published={pub} close={res} open->pub {1e6*(t1-t0):.0f}us "
              f"pub {1e6*(t2-t1):.0f}us close {1e6*(t3-t2):.0f}us", flush=True)
        torch.cuda.synchronize(dev)
        ctx.close()
