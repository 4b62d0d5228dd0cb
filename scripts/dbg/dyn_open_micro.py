"""Debug: host cost of the dynamic wave's calls (open / publish / close) and of the stream
handle lookup, on a 64-client ResNet-18 table (microseconds, medians over rounds)."""
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd._staging import NativeClientTable  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext  # noqa: E402

dev = torch.device("cuda", 0)
layout = resnet18_layout()
K = 64
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
ctx = FedAvgContext(layout, dev)
t = {"stream": [], "open": [], "publish4": [], "close": [], "sync": [], "query": []}
import ctypes  # noqa: E402
hip = ctypes.CDLL("libamdhip64.so")
for r in range(40):
    table = NativeClientTable(layout.num_segments, 0)
    for k in range(K):
        table.add_client(list(views[k]), [float(w[k])] * layout.num_segments)
    torch.cuda.synchronize()
    a = time.perf_counter(); s = ctx.stream; b = time.perf_counter(); t["stream"].append(b - a)
    a = time.perf_counter(); hip.hipStreamQuery(s); b = time.perf_counter(); t["query"].append(b - a)
    a = time.perf_counter(); ctx.dyn_open(torch.float32, 64); b = time.perf_counter(); t["open"].append(b - a)
    a = time.perf_counter(); ctx.dyn_publish(table); b = time.perf_counter(); t["publish4"].append(b - a)
    a = time.perf_counter(); ctx.dyn_close(None); b = time.perf_counter(); t["close"].append(b - a)
    a = time.perf_counter(); torch.cuda.synchronize(); b = time.perf_counter(); t["sync"].append(b - a)
    ctx.reset()
print({k: round(statistics.median(v[5:]) * 1e6, 1) for k, v in t.items()})
