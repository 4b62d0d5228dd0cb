"""How fast can a pageable host update (a ParameterMessage that came through a pipe) reach HBM?

Variants per client (ResNet-18 layout, fp32 and fp64, 62 tensors):
  to_device      : t.to(device) per tensor (pageable copy through HIP's internal staging)
  pinned_copy    : torch copy into a pinned flat buffer (one thread), then one async H2D
  pinned_copy_mt : the same host copy split over a thread pool, H2D on a copy stream
  host_register  : hipHostRegister the tensors' pages in place, async H2D, unregister
"""

from __future__ import annotations

import ctypes
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

from bench import resnet18_layout  # noqa: E402

dev = torch.device("cuda", 0)
layout = resnet18_layout()
P = layout.total_numel
N = 16
pool = ThreadPoolExecutor(8)
copy_stream = torch.cuda.Stream(dev)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]


def make_msgs(dtype):
    g = torch.Generator().manual_seed(1)
    msgs = []
    for _ in range(N):
        msgs.append({n: torch.randn(s, generator=g).to(dtype) for n, s in zip(layout.names, layout.shapes)})
    return msgs


def run(name, fn, msgs, nbytes):
    fn(msgs[:2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(msgs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"ms_per_client": round(dt / len(msgs) * 1e3, 3), "GBps": round(nbytes * len(msgs) / dt / 1e9, 2)}


def to_device(msgs):
    for m in msgs:
        for t in m.values():
            t.to(dev)


def make_pinned(msgs):
    esz = next(iter(msgs[0].values())).element_size()
    return [torch.empty(P, dtype=next(iter(msgs[0].values())).dtype).pin_memory() for _ in range(2)], esz


def pinned_copy_factory(mt):
    state = {}

    def fn(msgs):
        if "bufs" not in state:
            state["bufs"], _ = make_pinned(msgs)
            state["dev"] = [torch.empty(P, dtype=state["bufs"][0].dtype, device=dev) for _ in range(2)]
            state["ev"] = [None, None]
        for i, m in enumerate(msgs):
            b = i % 2
            if state["ev"][b] is not None:
                state["ev"][b].synchronize()  # the H2D that read this pinned buffer is done
            buf = state["bufs"][b]
            jobs = []
            o = 0
            for t in m.values():
                n = t.numel()
                if mt:
                    jobs.append(pool.submit(buf[o:o + n].copy_, t.view(-1)))
                else:
                    buf[o:o + n].copy_(t.view(-1))
                o += n
            for j in jobs:
                j.result()
            with torch.cuda.stream(copy_stream):
                state["dev"][b].copy_(buf, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            state["ev"][b] = ev

    return fn


def host_register(msgs):
    for m in msgs:
        regs = []
        for t in m.values():
            p, sz = t.data_ptr(), t.numel() * t.element_size()
            if hip.hipHostRegister(p, sz, 0) == 0:
                regs.append(p)
        with torch.cuda.stream(copy_stream):
            outs = [t.to(dev, non_blocking=True) for t in m.values()]
        copy_stream.synchronize()
        for p in regs:
            hip.hipHostUnregister(p)
        del outs


res = {}
for dtype in (torch.float32, torch.float64):
    msgs = make_msgs(dtype)
    nbytes = P * msgs[0]["fc.bias"].element_size()
    key = str(dtype).replace("torch.", "")
    res[key] = {
        "to_device": run("to_device", to_device, msgs, nbytes),
        "pinned_copy": run("pinned_copy", pinned_copy_factory(False), msgs, nbytes),
        "pinned_copy_mt": run("pinned_copy_mt", pinned_copy_factory(True), msgs, nbytes),
        "host_register": run("host_register", host_register, msgs, nbytes),
    }
    del msgs
print(json.dumps(res))
