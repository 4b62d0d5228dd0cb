"""PersonalizedFedAVG on one MI355X: every worker is a receiver (M = N), device-resident clients.

One step = one round of the reference's PersonalizedFedAVGAlgorithm
(personalized_aggregation_algorithm.py:23-57): N receivers' FedAvgs over the other N-1 updates
+ the centralized average, one HIP launch. Reports the kernel time (HIP events on the launch
stream), algorithmic bytes (N*P*s_in reads + (M+1)*P*s_out writes), algorithmic fp64 flops
(2 per folded (receiver, client, element) + 2 per centralized term), the measured fp64 VALU
ceiling and the measured HBM read ceiling.

    python scripts/bench_personalized.py --clients 64 --weights float
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from bench import LAYOUTS, hbm_probes  # noqa: E402
from distributed_learning_simulation_lib_amd.personalized import PersonalizedContext, fp64_probe  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet18", choices=sorted(LAYOUTS))
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--weights", default="float", choices=["float", "int"])
    ap.add_argument("--out-dtype", default="float64", choices=["float32", "float64"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-probe", action="store_true")
    args = ap.parse_args()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    layout = LAYOUTS[args.layout]()
    N = M = args.clients
    out_dtype = getattr(torch, args.out_dtype)
    P = layout.total_numel
    # clients: one flat bucket each, segments at 16-B aligned offsets, generated on the device
    offs, padded = layout.padded_offsets(4)
    g = torch.Generator(device=device).manual_seed(1234)
    clients = []
    for _ in range(N):
        b = torch.randn(padded, generator=g, device=device, dtype=torch.float32)
        clients.append([b[o : o + n] for o, n in zip(offs, layout.numels)])
    rng = np.random.default_rng(99)
    if args.weights == "int":
        w = rng.integers(100, 5001, size=(M, N)).astype(np.float64)
    else:
        w = rng.uniform(0.01, 3.0, size=(M, N))
    ooffs, opad = layout.padded_offsets(8)
    outs = []
    for _ in range(M):
        b = torch.empty(opad, dtype=out_dtype, device=device)
        outs.append([b[o : o + n] for o, n in zip(ooffs, layout.numels)])
    cb = torch.empty(opad, dtype=torch.float64, device=device)
    central = [cb[o : o + n] for o, n in zip(ooffs, layout.numels)]
    ctx = PersonalizedContext(layout, device)
    ids = list(range(N))

    tables = ctx.tables(clients, torch.float32, outs, out_dtype, central, torch.float64)  # persistent slots

    def step():
        ctx.aggregate(tables, torch.float32, ids, w, ids)

    for _ in range(args.warmup):
        step()
    assert ctx.check() == 0
    ctx.prof_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    flags = ctx.check()
    t1 = time.perf_counter()
    kms, launches = ctx.prof_collect()
    assert flags == 0
    ms_step = (t1 - t0) * 1e3 / args.steps
    kms_step = kms / args.steps
    s_out = torch.empty((), dtype=out_dtype).element_size()
    bytes_alg = N * P * 4 + M * P * s_out + P * 8
    folds = M * (N - 1) * P  # every receiver folds every other worker
    flops = 2 * folds + 2 * M * P
    res = {
        "workload": f"personalized_fedavg_{args.layout}_fp32_{N}x{M}",
        "clients": N, "receivers": M, "params_per_client": P, "tensors": layout.num_segments,
        "weights": args.weights, "out_dtype": args.out_dtype,
        "ms_per_step": round(ms_step, 4), "kernel_ms_per_step": round(kms_step, 4), "launches_per_step": launches // args.steps,
        "alg_bytes": bytes_alg, "kernel_GBps": round(bytes_alg / (kms_step * 1e-3) / 1e9, 1),
        "alg_fp64_flops": flops, "kernel_fp64_TFLOPs": round(flops / (kms_step * 1e-3) / 1e12, 2),
    }
    if not args.no_probe:
        res["fp64_fma_probe_TFLOPs"] = round(fp64_probe(device), 2)
        res["hbm_probe"] = hbm_probes(device)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
