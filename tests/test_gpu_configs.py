"""BASELINE configs 3 and 5 at full size on the one GPU, composed the way the ranks would run them.

config 3: 256 clients x ResNet-18 (11,689,512 fp32) sharded over 4 ranks (64 each);
config 5: 1024 clients x GPT-2 small (124,439,808 fp16) over 8 ranks (128 each), every shard
          streamed in waves of 32 through the fp64 accumulator.

Each shard runs the HIP partial kernel (zero-initialised, then continuing waves) exactly as its
rank would; the shards' fp64 partials are summed in rank order (the role of the RCCL reduce) and
finalized with the HIP finalize kernel. The client buffers of one shard are regenerated from the
global client seeds and reused (config 5 needs 255 GB of clients in total).

Checked on sampled elements (every segment's first and last element plus random ones):
  * bit-identical to the oracle's composition (each shard's arrival-order fp64 chain, the rank-
    order sum, / W, cast) — the kernels are exact;
  * within |Δ| <= 1e-12 * sum|w x| / W of the reference's single arrival-order chain
    (fed_avg_algorithm.py:43-99; the stated multi-GPU tolerance).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from bench import dataset_size_weights, gpt2s_layout, resnet18_layout
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext
from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer

pytestmark = pytest.mark.gpu


def _fill(buckets: torch.Tensor, first_client: int) -> None:
    """bench.make_clients' values: x ~ N(0,1), generator seeded 1234 + global client id."""
    g = torch.Generator(device=buckets.device)
    for i in range(buckets.shape[0]):
        g.manual_seed(1234 + first_client + i)
        buckets[i].normal_(generator=g)


def _samples(layout, rng, per_segment_random=40):
    """(segment, element) pairs: the ends of every segment and random interior elements."""
    picks = []
    for s, n in enumerate(layout.numels):
        picks += [(s, 0), (s, n - 1)]
        picks += [(s, int(i)) for i in rng.integers(0, n, size=min(per_segment_random, n))]
    return picks


def _run_sharded(layout, dtype, n_total, shards, wave, hip_device):
    T = layout.num_segments
    per = n_total // shards
    weights = dataset_size_weights(n_total)
    W = float(sum(weights))
    ctx = FedAvgContext(layout, hip_device)
    esize = torch.empty((), dtype=dtype).element_size()
    offs, padded = layout.padded_offsets(esize)
    picks = _samples(layout, np.random.default_rng(n_total))
    bucket_idx = torch.tensor([offs[s] + i for s, i in picks], device=hip_device)
    acc_idx = torch.tensor([ctx.segment_offset(s) + i for s, i in picks], device=hip_device)
    xs = np.empty((n_total, len(picks)), dtype=np.float64)
    summed = torch.zeros_like(ctx.accumulator)
    buckets = torch.empty((per, padded), dtype=dtype, device=hip_device)
    for r in range(shards):
        torch.cuda.synchronize(hip_device)  # the previous shard's kernels are done with the buffer
        _fill(buckets, r * per)
        tables = []
        for w0 in range(0, per, wave):
            table = ClientTable(T)
            for k in range(w0, min(per, w0 + wave)):
                row = [buckets[k, o : o + m] for o, m in zip(offs, layout.numels)]
                table.add_client(row, [weights[r * per + k]] * T)
            tables.append(table)
        # the rank's reducer: earlier waves folded into the accumulator, the last one as the
        # (chunkable) partial continuing from it
        red = HipLocalReducer(ctx, tables[-1], dtype, None, torch.float32, prior_waves=tables[:-1])
        red.prefold()
        red.partial(0, ctx.num_tiles)
        summed += ctx.accumulator  # rank-order sum of the shard partials (the reduce)
        xs[r * per : (r + 1) * per] = buckets[:, bucket_idx].double().cpu().numpy()
    ctx.accumulator.copy_(summed)
    ctx.set_accumulated([W] * T)
    out_offs, out_padded = layout.padded_offsets(4)
    flat = torch.empty(out_padded, dtype=torch.float32, device=hip_device)
    ctx.finalize_range([flat[o : o + m] for o, m in zip(out_offs, layout.numels)], torch.float32)
    ctx.raise_on_nan()
    got32 = flat[torch.tensor([out_offs[s] + i for s, i in picks], device=hip_device)].cpu().numpy()
    got_acc = ctx.accumulator[acc_idx].cpu().numpy()
    return xs, np.asarray(weights, dtype=np.float64), W, per, got32, got_acc


def _check(xs, w, W, per, got32, got_acc):
    n = xs.shape[0]
    # oracle composition: each shard's arrival-order chain, then the rank-order sum
    total = None
    for a in range(0, n, per):
        acc = xs[a] * w[a]
        for k in range(a + 1, a + per):
            acc = acc + xs[k] * w[k]
        total = acc if total is None else total + acc
    assert np.array_equal(got_acc.view(np.uint64), total.view(np.uint64))
    want = (total / W).astype(np.float32)
    assert np.array_equal(got32.view(np.uint32), want.view(np.uint32))
    # the reference's single chain, within the multi-GPU tolerance
    chain = xs[0] * w[0]
    for k in range(1, n):
        chain = chain + xs[k] * w[k]
    chain /= W
    mag = (np.abs(xs) * w[:, None]).sum(axis=0) / W
    assert np.all(np.abs(total / W - chain) <= 1e-12 * mag)
    ulp = np.spacing(np.abs(chain.astype(np.float32))).astype(np.float64)
    assert np.all(np.abs(got32.astype(np.float64) - chain.astype(np.float32).astype(np.float64)) <= ulp)


def test_config3_256_resnet18_fp32_as_4_shards(hip_device):
    xs, w, W, per, got32, got_acc = _run_sharded(resnet18_layout(), torch.float32, 256, 4, 64, hip_device)
    _check(xs, w, W, per, got32, got_acc)


def test_config5_1024_gpt2s_fp16_as_8_shards_in_waves(hip_device):
    xs, w, W, per, got32, got_acc = _run_sharded(gpt2s_layout(), torch.float16, 1024, 8, 32, hip_device)
    _check(xs, w, W, per, got32, got_acc)
    torch.cuda.empty_cache()
