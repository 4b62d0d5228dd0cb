"""Where FedAvgContext.aggregate's host time goes (GPU box): the Python pieces (table check,
arrays, output table, stream handle) and the native call, timed separately over many calls on an
8-client and a 64-client ResNet-18 table."""
from __future__ import annotations

import ctypes
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import _native, _staging  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext, OutputTable, dtype_code, out_code  # noqa: E402

R = 200
dev = torch.device("cuda", 0)
layout = resnet18_layout()
lib = _native.load()
for K in (8, 64):
    _, views = make_clients(layout, 0, K, dev, torch.float32)
    params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
    w = dataset_size_weights(K)
    index = {n: i for i, n in enumerate(layout.names)}
    shapes = [tuple(s) for s in layout.shapes]
    tab = _staging.NativeClientTable(layout.num_segments, 0)
    for p, x in zip(params, w):
        tab.rows.append(p, index, shapes, x, -1)
    ctx = FedAvgContext(layout, dev)
    offs, total = layout.padded_offsets(8)
    flat = torch.empty(total, dtype=torch.float64, device=dev)
    ot = OutputTable.from_flat(flat, offs, layout)
    t = {"check": 0.0, "arrays": 0.0, "out_table": 0.0, "stream": 0.0, "native": 0.0, "flags": 0.0}
    for r in range(R + 5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        ctx._check_table(tab, torch.float32)
        b = time.perf_counter()
        p, wv = tab.arrays()
        c = time.perf_counter()
        cat = ctx._out_table(ot, torch.float64)
        d = time.perf_counter()
        s = ctx.stream
        e = time.perf_counter()
        _native.check(lib.fedavg_aggregate(ctx._h, p.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)), dtype_code(torch.float32),
                                           wv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), K, cat,
                                           out_code(torch.float64), s))
        f = time.perf_counter()
        ctx.flags()
        g = time.perf_counter()
        ctx.reset()
        if r >= 5:
            for k, v in zip(t, (b - a, c - b, d - c, e - d, f - e, g - f)):
                t[k] += v
    print(json.dumps({"clients": K, **{k + "_us": round(v / R * 1e6, 2) for k, v in t.items()}}))
    ctx.close()
