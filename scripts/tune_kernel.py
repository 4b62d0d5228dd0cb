"""A/B the fused FedAvg kernel's compile-time knobs on the MI355X (one process, interleaved).

Usage (build here, run on the GPU box):
    python scripts/tune_kernel.py build     # compiles variants into distributed_learning_simulation_lib_amd/_lib/variants/
    python scripts/tune_kernel.py run       # on the GPU: 64 x ResNet-18 fp32 -> fp32, median kernel ms
"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

VARIANTS = {
    "base": {},
}
VDIR = REPO / "distributed_learning_simulation_lib_amd" / "_lib" / "variants"


def build_all():
    from distributed_learning_simulation_lib_amd.build import build

    for name, d in VARIANTS.items():
        print(name, build(defines=d or {"FEDAVG_VARIANT_BASE": 1}, out=VDIR / f"libfedavg_{name}.so"))


def run_all(rounds=7, iters=10):
    import numpy as np
    import torch

    from bench import dataset_size_weights, make_clients, resnet18_layout
    from distributed_learning_simulation_lib_amd import _native
    from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout, OutputTable

    dev = torch.device("cuda", 0)
    layout = resnet18_layout()
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    if len(sys.argv) > 3 and sys.argv[3] == "flat":
        layout = ModelLayout.flat(layout.total_numel)
    elif len(sys.argv) > 3 and sys.argv[3] != "resnet":
        from bench import LAYOUTS
        layout = LAYOUTS[sys.argv[3]]()
    dt = getattr(torch, sys.argv[4]) if len(sys.argv) > 4 else torch.float32
    buckets, views = make_clients(layout, 0, K, dev, dt)
    w = dataset_size_weights(K)
    wave = int(sys.argv[5]) if len(sys.argv) > 5 and int(sys.argv[5]) > 0 else K  # clients per launch (waves)
    tables = []
    for w0 in range(0, K, wave):
        t = ClientTable(layout.num_segments)
        for row, wk in zip(views[w0 : w0 + wave], w[w0 : w0 + wave]):
            t.add_client(row, [wk] * layout.num_segments)
        tables.append(t)
    table = tables[-1]

    class Waves:
        """aggregate() of the whole job: earlier waves accumulated, the last one fused."""

        def __init__(self, ctx):
            self.ctx = ctx

        def aggregate(self, _t, dt_, outs_, odt):
            for t in tables[:-1]:
                self.ctx.accumulate(t, dt_)
            self.ctx.aggregate(tables[-1], dt_, outs_, odt)
    offs, padded = layout.padded_offsets(4)
    flat = torch.empty(padded, dtype=torch.float32, device=dev)
    outs = OutputTable([flat[o:o + m] for o, m in zip(offs, layout.numels)], layout, dev, torch.float32)
    ctxs = {}
    ref = None
    for name in list(VARIANTS) + ["base_nofma"]:
        lib = _native.load(str(VDIR / f"libfedavg_{name.replace('_nofma', '')}.so"))
        ctxs[name] = FedAvgContext(layout, dev, lib=lib)
        if name.endswith("_nofma"):
            ctxs[name].set_fused_fold(False)
        Waves(ctxs[name]).aggregate(table, dt, outs, torch.float32)
        torch.cuda.synchronize()
        if ref is None:
            ref = flat.clone()
        if not name.startswith("abl"):
            assert torch.equal(ref.view(torch.int32), flat.view(torch.int32)), name
    times = {n: [] for n in ctxs}
    for _ in range(rounds):
        for name, ctx in ctxs.items():
            ctx.prof_enable(True)
            for _ in range(iters):
                Waves(ctx).aggregate(table, dt, outs, torch.float32)
            ctx.prof_enable(False)
            ms, n = ctx.prof_collect()
            times[name].append(ms / iters)  # kernel ms per job (all its launches)
    # algorithmic bytes of the job + the fp64 accumulator round trips between waves
    nbytes = K * layout.total_numel * buckets.element_size() + layout.total_numel * 4 \
        + (len(tables) - 1) * layout.total_numel * 16
    res = {}
    for name, t in times.items():
        med = float(np.median(t))
        res[name] = {"median_ms": round(med, 4), "min_ms": round(min(t), 4),
                     "GBps": round(nbytes / (med * 1e-3) / 1e9, 1)}
        print(f"{name:12s} median {med:.4f} ms  min {min(t):.4f}  {res[name]['GBps']} GB/s")
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build_all()
    else:
        run_all()
