"""BASELINE configs 2/4/5 at FULL size on one MI355X, checked on sampled elements.

The oracle cannot hold 44-255 GB on the host in seconds, so every element of the result is
produced by the kernel and a seeded sample of 200,000 element positions is re-computed by
the oracle from the very same client bytes (gathered on the GPU, folded on the host in the
same client order). Bit-exact, so any wrong tile, segment or client shows up.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from bench import dataset_size_weights, gpt2s_layout, make_clients, resnet18_layout, vitb16_layout
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, OutputTable
from oracle.fedavg_oracle import as_f64

pytestmark = pytest.mark.gpu
SAMPLE = 200_000


def _run(layout, K, dtype, hip_device, wave):
    buckets, views = make_clients(layout, 0, K, hip_device, dtype)
    w = dataset_size_weights(K)
    ctx = FedAvgContext(layout, hip_device)
    offs, padded = layout.padded_offsets(4)
    flat = torch.empty(padded, dtype=torch.float32, device=hip_device)
    outs = OutputTable([flat[o:o + m] for o, m in zip(offs, layout.numels)], layout, hip_device, torch.float32)
    for w0 in range(0, K, wave):
        t = ClientTable(layout.num_segments)
        for row, wk in zip(views[w0:w0 + wave], w[w0:w0 + wave]):
            t.add_client(row, [wk] * layout.num_segments)
        if w0 + wave < K:
            ctx.accumulate(t, dtype)
        else:
            ctx.aggregate(t, dtype, outs, torch.float32)
    ctx.raise_on_nan()
    # sampled positions in the padded client layout (same offsets for inputs of this dtype)
    in_offs, _ = layout.padded_offsets(buckets.element_size())
    rng = np.random.default_rng(K)
    seg = rng.integers(0, layout.num_segments, SAMPLE)
    pos = (rng.random(SAMPLE) * np.asarray(layout.numels)[seg]).astype(np.int64)
    idx_in = torch.from_numpy(np.asarray(in_offs)[seg] + pos).to(hip_device)
    idx_out = torch.from_numpy(np.asarray(offs)[seg] + pos).to(hip_device)
    xs = buckets[:, idx_in].cpu()  # [K, SAMPLE]
    got = flat[idx_out].cpu().numpy()
    if dtype == torch.bfloat16:
        xs64 = as_f64(xs.view(torch.int16).numpy().view(np.uint16), "bfloat16")
    else:
        xs64 = xs.numpy().astype(np.float64)
    acc = xs64[0] * w[0]
    for k in range(1, K):
        acc = acc + xs64[k] * w[k]
    want = (acc / float(sum(w))).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_config2_resnet18_64_clients(hip_device):
    _run(resnet18_layout(), 64, torch.float32, hip_device, wave=64)


def test_config4_vitb16_128_clients(hip_device):
    """128 x ViT-B/16 (152 tensors, 86.6 M params) fp32 = 44.3 GB resident, dataset-size weights."""
    _run(vitb16_layout(), 128, torch.float32, hip_device, wave=128)


def test_config5_gpt2s_fp16_waves(hip_device):
    """One GPU's share of config 5: 128 x GPT-2 small (148 tensors, 124.4 M params) fp16,
    folded in 4 waves of 32 through the fp64 accumulator."""
    _run(gpt2s_layout(), 128, torch.float16, hip_device, wave=32)
