#!/usr/bin/env python3
"""Headline benchmark: device-resident weighted FedAvg reduce on MI355X.

BASELINE.json metric: "aggregated GB/s (device-resident), N-client weighted FedAvg reduce,
1/2/4/8 GPU". One step = one full FedAvg aggregation of the resident client updates:

  N=1  (BASELINE config 2): 64 clients x ResNet-18 layout (62 tensors, 11,689,512 fp32
       params each), weights = client dataset sizes; one fused HIP launch folds the clients
       in fp64 and writes the fp32 global model; the NaN flag is read back (the reference's
       assertions) — the step ends when the host knows the round is valid.
  N>1  (BASELINE config 3 at N=4): weak scaling, 64 clients per GPU; every rank folds its
       shard into an fp64 partial, RCCL reduces the partials to rank 0 in chunks overlapped
       with the partial kernels, rank 0 finalizes each chunk as it lands.

value = algorithmic bytes of the whole job (all clients' reads + the output write) / step
time (max over ranks). Inputs are resident in HBM before the timed region. The
``roofline`` object prices the dominant kernel: algorithmic bytes per launch / its mean
duration from HIP events recorded on the launch stream inside the timed region. The
``cpu_baseline`` is the reference's CPU op sequence (oracle/ref_torch_cpu.py) on a bounded
sample of the same workload, rank 0, N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from distributed_learning_simulation_lib_amd.fedavg import (  # noqa: E402
    ClientTable,
    FedAvgContext,
    ModelLayout,
    OutputTable,
    bw_probe,
)
from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer, sharded_reduce  # noqa: E402

METRIC = "aggregated GB/s (device-resident), N-client weighted FedAvg reduce, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def resnet18_layout() -> ModelLayout:
    """torchvision ResNet-18 named_parameters(): 62 tensors, 11,689,512 elements."""
    shapes: list[tuple[str, tuple[int, ...]]] = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for b in range(2):
            pre = f"layer{li}.{b}"
            first_in = cin if b == 0 else cout
            shapes += [
                (f"{pre}.conv1.weight", (cout, first_in, 3, 3)),
                (f"{pre}.bn1.weight", (cout,)),
                (f"{pre}.bn1.bias", (cout,)),
                (f"{pre}.conv2.weight", (cout, cout, 3, 3)),
                (f"{pre}.bn2.weight", (cout,)),
                (f"{pre}.bn2.bias", (cout,)),
            ]
            if b == 0 and li > 1:
                shapes += [
                    (f"{pre}.downsample.0.weight", (cout, cin, 1, 1)),
                    (f"{pre}.downsample.1.weight", (cout,)),
                    (f"{pre}.downsample.1.bias", (cout,)),
                ]
        cin = cout
    shapes += [("fc.weight", (1000, 512)), ("fc.bias", (1000,))]
    layout = ModelLayout(names=tuple(n for n, _ in shapes), shapes=tuple(s for _, s in shapes))
    assert layout.num_segments == 62 and layout.total_numel == 11_689_512, layout.total_numel
    return layout


def dataset_size_weights(n: int, seed: int = 99) -> list[int]:
    rng = np.random.default_rng(seed)
    return [int(x) for x in rng.integers(100, 5001, size=n)]


def make_clients(layout: ModelLayout, first_client: int, n: int, device: torch.device, dtype: torch.dtype):
    """n synthetic client buckets x ~ N(0,1), seeded per global client id, resident in HBM."""
    offs, padded = layout.padded_offsets(torch.empty((), dtype=dtype).element_size())
    buckets = torch.empty((n, padded), dtype=dtype, device=device)
    g = torch.Generator(device=device)
    for i in range(n):
        g.manual_seed(1234 + first_client + i)
        buckets[i].normal_(generator=g)
    views = [[buckets[i, o : o + m] for o, m in zip(offs, layout.numels)] for i in range(n)]
    return buckets, views


def hbm_probes(device: torch.device, nbytes: int = 4 << 30) -> dict:
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    out = {}
    for mode, name, moved in ((0, "copy", 2 * nbytes), (1, "read", nbytes)):
        for _ in range(2):
            bw_probe(src, dst, mode)
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            bw_probe(src, dst, mode)
        e1.record()
        torch.cuda.synchronize(device)
        ms = e0.elapsed_time(e1) / reps
        out[f"{name}_GBps"] = round(moved / (ms * 1e-3) / 1e9, 1)
    del src, dst
    torch.cuda.empty_cache()
    return out


def cpu_baseline(layout: ModelLayout, budget_s: float = 12.0, sample_clients: int = 8) -> dict:
    """Reference CPU op sequence on a bounded sample of the same workload (rank 0, N=1)."""
    sys.path.insert(0, str(REPO))
    from oracle.ref_torch_cpu import RefOpsFedAvg

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    weights = dataset_size_weights(sample_clients)
    g = torch.Generator().manual_seed(1234)
    clients = [
        {n: torch.randn(s, generator=g, dtype=torch.float32) for n, s in zip(layout.names, layout.shapes)}
        for _ in range(sample_clients)
    ]
    nbytes = (sample_clients + 1) * layout.total_numel * 4
    times = []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s and len(times) < 1000:
        algo = RefOpsFedAvg()
        t0 = time.perf_counter()
        for c, w in zip(clients, weights):
            algo.add(c, w)
        out = algo.finish()
        out = {k: v.to(torch.float32) for k, v in out.items()}
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {
        "value": round(nbytes / best / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": (
            f"{sample_clients} clients x ResNet-18 layout fp32 (62 tensors, 11,689,512 params), "
            f"reference op sequence (isnan, to(f64)*w, +=, /W, isnan) in torch CPU, "
            f"best of {len(times)} runs over {time.perf_counter() - t_start:.1f} s"
        ),
    }


def committed_traffic(world: int, n_local: int, in_dtype: str, out_dtype: str) -> tuple[float | None, str | None]:
    """HBM bytes per launch of the same kernel and workload from the newest committed
    rocprofv3 PMC summary (scripts/profile.sh -> profiles/<tag>_traffic.json), or None."""
    if world != 1 or n_local != 64 or in_dtype != "float32" or out_dtype != "float32":
        return None, None
    files = sorted((REPO / "profiles").glob("r*_traffic.json"))
    if not files:
        return None, None
    d = json.loads(files[-1].read_text())
    return float(d["hbm_traffic_bytes_per_launch"]), f"profiles/{files[-1].name}"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clients-per-gpu", type=int, default=64)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--in-dtype", default="float32", choices=["float32", "float16", "bfloat16", "float64"])
    ap.add_argument("--out-dtype", default="float32", choices=["float32", "float64"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    in_dtype = getattr(torch, args.in_dtype)
    out_dtype = getattr(torch, args.out_dtype)
    layout = resnet18_layout()
    P = layout.total_numel
    n_local = args.clients_per_gpu
    n_total = n_local * world
    weights_all = dataset_size_weights(n_total)
    my_weights = weights_all[rank * n_local : (rank + 1) * n_local]

    buckets, views = make_clients(layout, rank * n_local, n_local, device, in_dtype)
    table = ClientTable(layout.num_segments)
    for row, w in zip(views, my_weights):
        table.add_client(row, [w] * layout.num_segments)
    ctx = FedAvgContext(layout, device)
    out_flat = None
    outs = None
    if rank == 0:
        offs, padded = layout.padded_offsets(torch.empty((), dtype=out_dtype).element_size())
        out_flat = torch.empty(padded, dtype=out_dtype, device=device)
        outs = OutputTable([out_flat[o : o + m] for o, m in zip(offs, layout.numels)], layout, device, out_dtype)
    reducer = HipLocalReducer(ctx, table, in_dtype, outs, out_dtype)
    local_totals = [float(sum(my_weights))] * layout.num_segments
    global_totals = [float(sum(weights_all))] * layout.num_segments

    def step() -> None:
        sharded_reduce(reducer, local_totals, chunks=args.chunks, global_total_weights=global_totals)
        if rank == 0:
            ctx.raise_on_nan()  # the reference's assertions: the round ends on the host

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    ctx.prof_collect()  # drop warmup events
    ctx.prof_enable(True)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    ctx.prof_enable(False)
    kernel_ms, launches = ctx.prof_collect()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    in_bytes = np.dtype(np.float32).itemsize if in_dtype == torch.float32 else torch.empty((), dtype=in_dtype).element_size()
    out_bytes = torch.empty((), dtype=out_dtype).element_size()
    job_bytes = n_total * P * in_bytes + P * out_bytes
    step_s = elapsed / args.steps
    value_gbps = job_bytes / step_s / 1e9

    # dominant kernel: N=1 -> the fused launch (clients read + output write);
    # N>1 -> this rank's launches per step (partial chunks + finalize on root)
    per_launch_ms = kernel_ms / max(launches, 1)
    if world == 1:
        launch_bytes = n_local * P * in_bytes + P * out_bytes
        kernel_s = per_launch_ms * 1e-3
    else:
        launch_bytes = n_local * P * in_bytes + P * 8  # this rank's fp64 partial write
        kernel_s = kernel_ms * 1e-3 / args.steps
    achieved = launch_bytes / kernel_s / 1e9 if kernel_s > 0 else 0.0

    traffic, traffic_src = committed_traffic(world, n_local, args.in_dtype, args.out_dtype)
    probe = None
    cpu = None
    if rank == 0 and not args.no_probe:
        probe = hbm_probes(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del buckets, views, table, reducer
        torch.cuda.empty_cache()
        cpu = cpu_baseline(layout)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return 0
    line = {
        "metric": METRIC,
        "value": round(value_gbps, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: client params ~ N(0,1) seeded per client, weights = dataset sizes in [100, 5000]",
        "config": {
            "workload": "fedavg_resnet18_fp32_64_clients_per_gpu",
            "clients_per_gpu": n_local,
            "total_clients": n_total,
            "params_per_client": P,
            "tensors_per_client": layout.num_segments,
            "in_dtype": args.in_dtype,
            "accumulate_dtype": "float64",
            "out_dtype": args.out_dtype,
            "parallelism": "single GPU" if world == 1 else f"clients sharded over {world} GPUs + chunked RCCL reduce to rank 0",
            "baseline_config": "BASELINE.json configs[1]" if world == 1 else "BASELINE.json configs[2] (weak-scaled, 64 clients/GPU)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "fedavg_tile_kernel<float, OUT_F32, 1, true>" if world == 1 else "fedavg_tile_kernel<float, OUT_ACC, 1, true> (+finalize)",
            "bytes_per_launch": launch_bytes,
            "mean_launch_ms": round(per_launch_ms, 4),
            "launches": launches,
        },
        "hbm_probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
