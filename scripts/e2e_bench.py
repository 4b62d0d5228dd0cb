"""End-to-end FedAvg rate with client updates arriving in HOST memory (GPU box).

The headline bench is device-resident; the reference's updates arrive as CPU tensors from
worker processes (aggregation_worker.py:152, aggregation_server.py:129). This measures a
whole round from host payloads to the host copy of the global model, for 64 clients x the
ResNet-18 layout:

  plugin_pageable_fp32 : FedAVGAlgorithm.process_worker_data on 64 pageable CPU fp32 messages
                         (62 tensors each; each tensor moved to the GPU as it is staged),
                         aggregate_worker_data, result copied to the host as float64 (what the
                         reference server caches, util/model_cache.py:27-34)
  plugin_pageable_fp64 : the same with float64 payloads (what AggregationWorker sends)
  plugin_pageable_qsgd255: the same with QSGD-quantised payloads (level 255; records staged
                         through the pinned ingest, dequantised inside the fold)
  pinned_pipelined_fp32: payloads in pinned host buckets; H2D copies on a copy stream, one
                         accumulate launch per wave of 8 clients as soon as its copies land,
                         fp64 result D2H

GB/s = algorithmic bytes (client payload bytes + one result write) / round wall time.
"""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from bench import dataset_size_weights, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, OutputTable  # noqa: E402

K = 64
dev = torch.device("cuda", 0)
layout = resnet18_layout()
P = layout.total_numel
w = dataset_size_weights(K)
results = {}


def host_clients(dtype, pinned):
    g = torch.Generator().manual_seed(5)
    base = torch.randn(P, generator=g).to(dtype)
    out = []
    for k in range(K):
        flat = (base * (1.0 + k / K)).to(dtype)
        if pinned:
            flat = flat.pin_memory()
        offs = 0
        d = {}
        for n, s in zip(layout.names, layout.shapes):
            m = int(torch.Size(s).numel())
            d[n] = flat[offs:offs + m].view(s)
            offs += m
        out.append((flat, d))
    return out


def plugin_round(clients):
    algo = FedAVGAlgorithm(device=dev, wave_size=64, result_device="cpu")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, (_, d) in enumerate(clients):
        algo.process_worker_data(k, ParameterMessage(parameter=dict(d), aggregation_weight=w[k]))
    res = algo.aggregate_worker_data()
    host = res.parameter  # result_device="cpu": one D2H copy of the flat result
    dt = time.perf_counter() - t0
    algo.exit()
    assert all(v.dtype == torch.float64 for v in host.values())
    return dt


for dtype, name in ((torch.float32, "plugin_pageable_fp32"), (torch.float64, "plugin_pageable_fp64")):
    clients = host_clients(dtype, pinned=False)
    plugin_round(clients)  # warm
    times = [plugin_round(clients) for _ in range(3)]
    nbytes = K * P * clients[0][0].element_size() + P * 8
    results[name] = {"round_ms": round(min(times) * 1e3, 2), "GBps": round(nbytes / min(times) / 1e9, 2)}
    del clients

# QSGD-quantised updates in host memory (StochasticQuantServerEndpoint): the plugin stages the
# records (1.125 B/element) through the pinned ingest and the kernel dequantises in the fold
from distributed_learning_simulation_lib_amd.quantized import quantize_tensor  # noqa: E402

dense = host_clients(torch.float32, pinned=False)
qclients = []
gq = torch.Generator(device=dev).manual_seed(11)
for flat, d in dense:
    qd = {n: quantize_tensor(t.to(dev), generator=gq).to("cpu") for n, t in d.items()}
    qclients.append((None, qd))
del dense
plugin_round(qclients)  # warm
times = [plugin_round(qclients) for _ in range(3)]
rec_bytes = sum(q.record.numel() for q in qclients[0][1].values())
results["plugin_pageable_qsgd255"] = {
    "round_ms": round(min(times) * 1e3, 2),
    "GBps": round((K * rec_bytes + P * 8) / min(times) / 1e9, 2),
    "fp32_equivalent_GBps": round((K * P * 4 + P * 8) / min(times) / 1e9, 2),
}
del qclients

# pinned, pipelined H2D (copy stream) + per-wave accumulate on the compute stream
clients = host_clients(torch.float32, pinned=True)
WAVE = 8
staging = [torch.empty(P, dtype=torch.float32, device=dev) for _ in range(2 * WAVE)]
ctx = FedAvgContext(layout, dev)
offs, padded = layout.padded_offsets(8)
res_flat = torch.empty(padded, dtype=torch.float64, device=dev)
outs = OutputTable([res_flat[o:o + m] for o, m in zip(offs, layout.numels)], layout, dev, torch.float64)
host_res = torch.empty(padded, dtype=torch.float64).pin_memory()
copy_stream = torch.cuda.Stream(dev)


def pipelined_round():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ready = []
    comp = torch.cuda.current_stream(dev)
    for wv in range(K // WAVE):
        bank = (wv % 2) * WAVE
        ev_free = torch.cuda.Event()
        ev_free.record(comp)  # the compute stream finished reading this bank two waves ago
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(ev_free)
            for j in range(WAVE):
                staging[bank + j].copy_(clients[wv * WAVE + j][0], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(copy_stream)
        ready.append(ev)
        comp.wait_event(ev)
        table = ClientTable(layout.num_segments)
        for j in range(WAVE):
            flat = staging[bank + j]
            row, o = [], 0
            for m in layout.numels:
                row.append(flat[o:o + m])
                o += m
            table.add_client(row, [w[wv * WAVE + j]] * layout.num_segments)
        if wv < K // WAVE - 1:
            ctx.accumulate(table, torch.float32)
        else:
            ctx.aggregate(table, torch.float32, outs, torch.float64)
    ctx.raise_on_nan()
    host_res.copy_(res_flat, non_blocking=True)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


pipelined_round()
times = [pipelined_round() for _ in range(3)]
results["pinned_pipelined_fp32"] = {"round_ms": round(min(times) * 1e3, 2),
                                    "GBps": round((K * P * 4 + P * 8) / min(times) / 1e9, 2)}
print(json.dumps({"workload": "64 clients x ResNet-18 (11,689,512 params), host payloads -> host fp64 model",
                  "results": results}))
